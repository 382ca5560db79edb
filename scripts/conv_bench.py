#!/usr/bin/env python3
"""Per-layer A/B of the implicit-GEMM convolution kernels (csrc/conv_igemm.hip) against MIOpen
on every ResNet-50 convolution shape: numerics (vs an fp32 reference of the same bf16 inputs),
then forward and stride-1 input-gradient timings at the benchmark batch, one JSON line per shape.

    python scripts/conv_bench.py [--batch 512] [--only fwd|dgrad] [--out gpurun_out/conv_bench.jsonl]
"""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(ROOT, "determined_amd", "benchmarks", "miopen_db"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

# (cin, cout, k, stride, input hw, count in ResNet-50)
SHAPES = [
    (64, 64, 1, 1, 56, 1), (64, 64, 3, 1, 56, 3), (64, 256, 1, 1, 56, 4), (256, 64, 1, 1, 56, 2),
    (256, 128, 1, 1, 56, 1), (128, 128, 3, 2, 56, 1), (128, 512, 1, 1, 28, 4), (256, 512, 1, 2, 56, 1),
    (512, 128, 1, 1, 28, 3), (128, 128, 3, 1, 28, 3),
    (512, 256, 1, 1, 28, 1), (256, 256, 3, 2, 28, 1), (256, 1024, 1, 1, 14, 6), (512, 1024, 1, 2, 28, 1),
    (1024, 256, 1, 1, 14, 5), (256, 256, 3, 1, 14, 5),
    (1024, 512, 1, 1, 14, 1), (512, 512, 3, 2, 14, 1), (512, 2048, 1, 1, 7, 3), (1024, 2048, 1, 2, 14, 1),
    (2048, 512, 1, 1, 7, 2), (512, 512, 3, 1, 7, 2),
]


def timeit(fn, iters=10, reps=3):
    fn()
    torch.cuda.synchronize()
    best = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        best.append(s.elapsed_time(e) * 1000.0 / iters)
    best.sort()
    return best[len(best) // 2]


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--only", default="")
    ap.add_argument("--shapes", default="", help="comma list of shape indices")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    from determined_amd import ops
    e = ops.ext()
    ncfg = e.conv_num_cfgs()
    dev = torch.device("cuda")
    out = open(a.out, "a") if a.out else None
    idx = [int(i) for i in a.shapes.split(",")] if a.shapes else range(len(SHAPES))
    tot = {"miopen_fwd": 0.0, "ours_fwd": 0.0, "miopen_dgrad": 0.0, "ours_dgrad": 0.0, "miopen_wgrad": 0.0,
           "ours_wgrad": 0.0}
    for si in idx:
        cin, cout, k, st, hw, cnt = SHAPES[si]
        pad = k // 2
        rec = {"cin": cin, "cout": cout, "k": k, "stride": st, "hw": hw, "count": cnt}
        # ---- numerics at a small batch
        torch.manual_seed(si)
        xs = cl(torch.randn(3, cin, hw, hw, device=dev).to(torch.bfloat16))
        w = cl((torch.randn(cout, cin, k, k, device=dev) / (cin * k * k) ** 0.5).to(torch.bfloat16))
        ref = F.conv2d(xs.float(), w.float(), stride=st, padding=pad)
        errs = {}
        for cfg in range(ncfg):
            if not e.conv_supported(xs, w, cfg, st, pad):
                continue
            y, part = e.conv_fwd(xs, w, st, pad, True, cfg, 0)
            err = ((y.float() - ref).norm() / ref.norm()).item()
            ssum = ref.sum((0, 2, 3))  # the epilogue sums the fp32 outputs
            ssq = (ref * ref).sum((0, 2, 3))
            serr = max(((part[:, 0].sum(0) - ssum).abs().max() / ssum.abs().max().clamp_min(1e-3)).item(),
                       ((part[:, 1].sum(0) - ssq).abs().max() / ssq.abs().max()).item())
            errs[cfg] = (round(err, 5), round(serr, 6))
        rec["rel_err"] = {str(c): v for c, v in errs.items()}
        # ---- timing at the benchmark batch
        x = cl(torch.randn(a.batch, cin, hw, hw, device=dev).to(torch.bfloat16))
        oh = (hw + 2 * pad - k) // st + 1
        if a.only in ("", "fwd"):
            rec["miopen_fwd_us"] = round(timeit(lambda: F.conv2d(x, w, stride=st, padding=pad)), 1)
            rec["ours_fwd_us"] = {}
            for cfg in errs:
                rec["ours_fwd_us"][str(cfg)] = round(timeit(lambda: e.conv_fwd(x, w, st, pad, False, cfg, 0)), 1)
            rec["ours_fwd_stats_us"] = {}
            for cfg in errs:
                rec["ours_fwd_stats_us"][str(cfg)] = round(timeit(lambda: e.conv_fwd(x, w, st, pad, True, cfg, 0)), 1)
            best = min(rec["ours_fwd_stats_us"].values())
            tot["miopen_fwd"] += rec["miopen_fwd_us"] * cnt
            tot["ours_fwd"] += min(best, rec["miopen_fwd_us"]) * cnt
            rec["roofline_fwd_us"] = round((x.numel() + a.batch * cout * oh * oh) * 2 / 6.0e6, 1)
            rec["flop_floor_us"] = round(2.0 * a.batch * oh * oh * cout * cin * k * k / 2.0e9, 1)
        if a.only in ("", "dgrad") and st == 1:
            dy = cl(torch.randn(a.batch, cout, hw, hw, device=dev).to(torch.bfloat16))
            wt = cl(w.flip(2, 3).transpose(0, 1))

            def miopen_dgrad():
                return torch.ops.aten.convolution_backward(dy, x, w, None, [st, st], [pad, pad], [1, 1], False, [0, 0],
                                                           1, [True, False, False])[0]
            rec["miopen_dgrad_us"] = round(timeit(miopen_dgrad), 1)
            rec["ours_dgrad_us"] = {}
            for cfg in range(ncfg):
                if e.conv_supported(dy, wt, cfg, 1, k - 1 - pad):
                    rec["ours_dgrad_us"][str(cfg)] = round(timeit(lambda: e.conv_fwd(dy, wt, 1, k - 1 - pad, False, cfg, 0)), 1)
            if rec["ours_dgrad_us"]:
                tot["miopen_dgrad"] += rec["miopen_dgrad_us"] * cnt
                tot["ours_dgrad"] += min(min(rec["ours_dgrad_us"].values()), rec["miopen_dgrad_us"]) * cnt
        if a.only in ("", "wgrad"):
            dyw = cl(torch.randn(a.batch, cout, oh, oh, device=dev).to(torch.bfloat16))

            def miopen_wgrad():
                return torch.ops.aten.convolution_backward(dyw, x, w, None, [st, st], [pad, pad], [1, 1], False,
                                                           [0, 0], 1, [False, True, False])[1]
            rec["miopen_wgrad_us"] = round(timeit(miopen_wgrad), 1)
            dys = cl(torch.randn(3, cout, oh, oh, device=dev).to(torch.bfloat16))
            refw = torch.nn.grad.conv2d_weight(xs.float(), w.shape, dys.float(), stride=st, padding=pad)
            rec["ours_wgrad_us"] = {}
            rec["wgrad_err"] = {}
            for cfg in range(e.wgrad_num_cfgs()):
                if e.wgrad_supported(x, dyw, cout, cfg):
                    got = e.conv_wgrad(xs, dys, w, st, pad, cfg, 0).float()
                    rec["wgrad_err"][str(cfg)] = round(((got - refw).norm() / refw.norm()).item(), 5)
                    rec["ours_wgrad_us"][str(cfg)] = round(timeit(lambda: e.conv_wgrad(x, dyw, w, st, pad, cfg, 0)), 1)
            if k == 3 and st == 1:  # 3x3 halo weight gradient
                for c in (0, 1):
                    if e.wgrad3x3_supported(x, dyw, w, c):
                        got = e.conv3x3_wgrad(xs, dys, w, c, 0).float()
                        rec["wgrad_err"][f"h{c}"] = round(((got - refw).norm() / refw.norm()).item(), 5)
                        rec["ours_wgrad_us"][f"h{c}"] = round(timeit(lambda: e.conv3x3_wgrad(x, dyw, w, c, 0)), 1)
            if rec["ours_wgrad_us"]:
                tot["miopen_wgrad"] += rec["miopen_wgrad_us"] * cnt
                tot["ours_wgrad"] += min(min(rec["ours_wgrad_us"].values()), rec["miopen_wgrad_us"]) * cnt
        line = json.dumps(rec)
        print(line, flush=True)
        if out:
            out.write(line + "\n")
            out.flush()
    line = json.dumps({"batch": a.batch, "totals_us_weighted": {k: round(v, 1) for k, v in tot.items()}})
    print(line, flush=True)
    if out:
        out.write(line + "\n")


if __name__ == "__main__":
    main()
