#!/usr/bin/env python3
"""Time the stride-2 3x3 input gradient: MIOpen vs the four-phase implicit-GEMM kernels (per tile
config), on ResNet-50's three stride-2 3x3 convs at the benchmark batch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from determined_amd import ops  # noqa: E402
from determined_amd.ops import conv as C  # noqa: E402

e = ops.ext()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024


def t(fn):
    fn()
    ts = []
    for _ in range(5):
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(5):
            fn()
        s1.record()
        s1.synchronize()
        ts.append(s0.elapsed_time(s1) * 200.0)
    return sorted(ts)[2]


for ch, hw in ((128, 56), (256, 28), (512, 14)):
    w = (torch.randn(ch, ch, 3, 3, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x = torch.empty(B, ch, hw, hw, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(B, ch, hw // 2, hw // 2, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    mi = lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1,  # noqa
                                                     [True, False, False])[0]
    ref = mi()
    out = [f"{ch}ch {hw}x{hw}: miopen {t(mi):.1f} us"]
    for c in C._phase_cfgs(e, dy, w):
        fn = lambda c=c: C._dgrad_s2_phases(e, dy, w, x.shape, c)  # noqa: E731
        err = ((fn().float() - ref.float()).norm() / ref.float().norm()).item()
        out.append(f"p{c} {t(fn):.1f} us (err {err:.1e})")
    print("; ".join(out), flush=True)
