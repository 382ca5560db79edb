#!/usr/bin/env python3
"""Per-layer roofline table of ResNet-50's convolutions on the kernels the model actually picks.

For every bottleneck conv shape (scripts/conv_bench.py SHAPES) at the benchmark batch: the forward
(with the BN-statistics epilogue, ``ops.conv.conv_bn_input``), the input gradient
(``ops.conv._dgrad``) and the weight gradient (``ops.conv._wgrad``) are tuned exactly as in
training (per-layer timed choice), then timed.  Each gets its FLOP floor (at ``--pflops``) and its
byte floor (operands read once + result written once, at ``--tbs``); the table shows the achieved
rate, the floor, and the fraction of the step spent above the floor, weighted by how often the
shape occurs in the network.  One JSON line per (shape, pass), then a summary.

    python scripts/layer_roofline.py [--batch 1024] [--out gpurun_out/layer_roofline.jsonl]
"""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(ROOT, "determined_amd", "benchmarks", "miopen_db"))

import torch  # noqa: E402
from torch import nn  # noqa: E402

from conv_bench import SHAPES, timeit  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--pflops", type=float, default=2.0, help="bf16 MFMA rate the floor assumes (PFLOP/s)")
    ap.add_argument("--tbs", type=float, default=6.0, help="HBM rate the floor assumes (TB/s)")
    ap.add_argument("--out", default="gpurun_out/layer_roofline.jsonl")
    a = ap.parse_args()
    from determined_amd import ops
    from determined_amd.ops import conv as C

    ops.ext()
    cl = torch.channels_last
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    out = open(a.out, "w")
    tot = {"fwd": [0.0, 0.0], "dgrad": [0.0, 0.0], "wgrad": [0.0, 0.0]}
    for cin, cout, k, st, hw, cnt in SHAPES:
        pad = k // 2
        oh = (hw + 2 * pad - k) // st + 1
        n = a.batch
        x = torch.randn(n, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        conv = nn.Conv2d(cin, cout, k, stride=st, padding=pad, bias=False).cuda().to(torch.bfloat16)
        conv = conv.to(memory_format=cl)
        w = conv.weight.detach()
        dy = torch.randn(n, cout, oh, oh, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        m = n * oh * oh
        flops = 2.0 * m * cout * cin * k * k
        bx, by, bw = x.numel() * 2, dy.numel() * 2, w.numel() * 2
        passes = {
            "fwd": (lambda: C.conv_bn_input(conv, x), bx + bw + by),
            "dgrad": (lambda: C._dgrad(dy, x, w, st, pad), by + bw + bx),
            "wgrad": (lambda: C._wgrad(dy, x, w, st, pad), bx + by + bw),
        }
        for name, (fn, nbytes) in passes.items():
            with torch.no_grad():
                us = timeit(fn)
            t_flop = flops / (a.pflops * 1e15) * 1e6
            t_byte = nbytes / (a.tbs * 1e12) * 1e6
            floor = max(t_flop, t_byte)
            key = {"fwd": ("fwd", tuple(x.shape), tuple(w.shape), st, pad),
                   "dgrad": ("dgrad", tuple(dy.shape), tuple(w.shape), st, pad),
                   "wgrad": ("wgrad", tuple(x.shape), tuple(w.shape), st, pad)}[name]
            rec = {"cin": cin, "cout": cout, "k": k, "stride": st, "hw": hw, "count": cnt, "pass": name,
                   "us": round(us, 1), "floor_us": round(floor, 1), "bound": "flop" if t_flop >= t_byte else "byte",
                   "tflops": round(flops / us / 1e6, 1), "tbs": round(nbytes / us / 1e6, 2),
                   "frac_of_floor": round(floor / us, 3), "choice": C.tuned_choices().get(key)}
            tot[name][0] += us * cnt
            tot[name][1] += floor * cnt
            out.write(json.dumps(rec) + "\n")
            out.flush()
            print(f"{cin:5d}->{cout:5d} k{k} s{st} {hw:3d}x{cnt}  {name:5s} {us:8.1f}us floor {floor:7.1f} "
                  f"({rec['bound']}) {rec['tflops']:6.1f} TF/s {rec['tbs']:5.2f} TB/s  choice={rec['choice']}",
                  flush=True)
        del x, dy, conv, w
        torch.cuda.empty_cache()
    summ = {p: {"ms": round(v[0] / 1e3, 2), "floor_ms": round(v[1] / 1e3, 2)} for p, v in tot.items()}
    out.write(json.dumps({"batch": a.batch, "summary": summ}) + "\n")
    print(json.dumps({"batch": a.batch, "summary": summ}))


if __name__ == "__main__":
    main()
