#!/usr/bin/env python3
"""HBM bandwidth of the standalone BN apply passes at the bench batch (bf16 NHWC): the forward apply
(y = relu(x*s + h)) and the deferred backward apply (dx = A dz + B y + C) on the ResNet-50 shapes the
per-layer choice leaves unfused.  One JSON line per (pass, shape): us and TB/s of compulsory traffic.

    python scripts/bn_apply_bw.py [--batch 2048]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("DAMD_AB_ROOT", ROOT))  # A/B: another build of the package
import torch  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    t.record()
    t.synchronize()
    return s.elapsed_time(t) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    a = ap.parse_args()
    from determined_amd import ops

    e = ops.ext()
    for hw, c in ((56, 256), (28, 512), (14, 1024), (56, 64), (28, 128), (14, 256)):
        x = torch.randn(a.batch, c, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = torch.randn_like(x)
        coef = torch.randn(3, c, device="cuda").contiguous()
        sc, sh = torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda")
        nbytes = x.numel() * 2
        us = timeit(lambda: e.bn_bwd_apply_coef(x, y, coef))
        print(json.dumps({"pass": "bn_bwd_apply", "hw": hw, "c": c, "batch": a.batch, "us": round(us, 1),
                          "tbs": round(3 * nbytes / us / 1e6, 2)}), flush=True)
        us = timeit(lambda: e.bn_apply(x, sc, sh, None, True))
        print(json.dumps({"pass": "bn_apply", "hw": hw, "c": c, "batch": a.batch, "us": round(us, 1),
                          "tbs": round(2 * nbytes / us / 1e6, 2)}), flush=True)
        del x, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
