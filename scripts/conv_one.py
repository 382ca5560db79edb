#!/usr/bin/env python3
"""Run one implicit-GEMM conv launch config repeatedly (for rocprofv3 PMC passes).

    python scripts/conv_one.py CIN COUT K STRIDE HW CFG [--batch 512] [--iters 20] [--mode fwd|dgrad_bn_pro|wgrad3x3]

``--mode wgrad3x3``: the 3x3 stride-1 weight gradient, CFG = wgrad3x3 config (0/1 conv_igemm.hip, 2.. conv3x3v2.hip).
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
ap.add_argument("--mode", default="fwd", choices=["fwd", "dgrad_bn_pro", "wgrad3x3"])
a = ap.parse_args()
from determined_amd import ops  # noqa: E402

e = ops.ext()
cl = torch.channels_last
x = torch.randn(a.batch, a.cin, a.hw, a.hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
w = torch.randn(a.cout, a.cin, a.k, a.k, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
pad = a.k // 2
if a.mode == "wgrad3x3":
    dy = torch.randn(a.batch, a.cout, a.hw, a.hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    assert a.k == 3 and a.stride == 1 and e.wgrad3x3_supported(x, dy, w, a.cfg)
    for _ in range(a.iters):
        e.conv3x3_wgrad(x, dy, w, a.cfg, 0)
    torch.cuda.synchronize()
    print("ok")
    sys.exit(0)
assert e.conv_supported(x, w, a.cfg, a.stride, pad)
if a.mode == "dgrad_bn_pro":
    # 1x1 input gradient of a chained ResNet block: operand dy = A*dz + B*y + Cc formed in the
    # staging (x = dz, yn = y), BN-backward epilogue with the ReLU bit mask and the shortcut gradient
    assert a.k == 1 and a.stride == 1 and e.conv_pro_supported(x, w, a.cfg)
    yn = torch.randn_like(x)
    coef = torch.randn(3, a.cin, device="cuda").contiguous()
    yb = torch.randn(a.batch, a.cout, a.hw, a.hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    res = torch.randn_like(yb)
    _, stats, mask = e.bn_act_fwd(yb, torch.rand(a.cout, device="cuda") + 0.5, torch.randn(a.cout, device="cuda"),
                                  None, None, 0.0, 1e-5, res, True, True, None)
    d2 = torch.randn_like(yb)
    for _ in range(a.iters):
        e.conv_dgrad_bn(x, w, 0, a.cfg, d2, yb, mask, stats, yn, coef)
else:
    for _ in range(a.iters):
        e.conv_fwd(x, w, a.stride, pad, True, a.cfg, 0)
torch.cuda.synchronize()
print("ok")
