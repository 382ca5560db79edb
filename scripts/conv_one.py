#!/usr/bin/env python3
"""Run one implicit-GEMM conv launch config repeatedly (for rocprofv3 PMC passes).

    python scripts/conv_one.py CIN COUT K STRIDE HW CFG [--batch 512] [--iters 20] [--mode fwd|dgrad_bn]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

ap = argparse.ArgumentParser()
for n in ("cin", "cout", "k", "stride", "hw", "cfg"):
    ap.add_argument(n, type=int)
ap.add_argument("--batch", type=int, default=512)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
from determined_amd import ops  # noqa: E402

e = ops.ext()
cl = torch.channels_last
x = torch.randn(a.batch, a.cin, a.hw, a.hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
w = torch.randn(a.cout, a.cin, a.k, a.k, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
pad = a.k // 2
assert e.conv_supported(x, w, a.cfg, a.stride, pad)
for _ in range(a.iters):
    e.conv_fwd(x, w, a.stride, pad, True, a.cfg, 0)
torch.cuda.synchronize()
print("ok")
