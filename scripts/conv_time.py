#!/usr/bin/env python3
"""Time implicit-GEMM conv configs on one layer shape (median of repeated launches).

    python scripts/conv_time.py CIN COUT K STRIDE HW CFG[,CFG...] [--batch 1024] [--stats]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

ap = argparse.ArgumentParser()
for n in ("cin", "cout", "k", "stride", "hw"):
    ap.add_argument(n, type=int)
ap.add_argument("cfgs")
ap.add_argument("--batch", type=int, default=1024)
ap.add_argument("--stats", action="store_true")
a = ap.parse_args()
from determined_amd import ops  # noqa: E402

e = ops.ext()
cl = torch.channels_last
x = torch.randn(a.batch, a.cin, a.hw, a.hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
w = (torch.randn(a.cout, a.cin, a.k, a.k, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
pad = a.k // 2
# fp32 reference in batch chunks: a single fp32 conv over >4 GiB tensors is not trustworthy here.
ref = torch.cat([torch.nn.functional.conv2d(xc.float(), w.float(), stride=a.stride, padding=pad)
                 for xc in x.split(256)]).to(torch.bfloat16)


def rel_err(y):
    num = den = 0.0
    for yc, rc in zip(y.split(256), ref.split(256)):
        num += (yc.float() - rc.float()).norm().item() ** 2
        den += rc.float().norm().item() ** 2
    return (num / den) ** 0.5


for c in (int(v) for v in a.cfgs.split(",")):
    if not e.conv_supported(x, w, c, a.stride, pad):
        print(f"cfg {c}: unsupported")
        continue
    y = e.conv_fwd(x, w, a.stride, pad, a.stats, c, 0)[0]
    err = rel_err(y)
    ts = []
    for _ in range(5):
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(10):
            e.conv_fwd(x, w, a.stride, pad, a.stats, c, 0)
        s1.record()
        s1.synchronize()
        ts.append(s0.elapsed_time(s1) * 100.0)
    ts.sort()
    flops = 2.0 * a.batch * (a.hw // a.stride) ** 2 * a.cout * a.cin * a.k * a.k
    print(f"{a.cin}->{a.cout} k{a.k} s{a.stride} {a.hw} cfg {c}: {ts[2]:.1f} us ({flops / ts[2] / 1e6:.0f} TF/s) "
          f"rel_err {err:.2e}", flush=True)
