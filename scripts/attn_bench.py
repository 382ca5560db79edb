#!/usr/bin/env python3
"""Flash attention micro-benchmark: our MFMA kernel vs PyTorch SDPA (fwd, fwd+bwd), GPT-2 shapes."""
import json
import math
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from determined_amd.ops.attention import flash_attention  # noqa: E402


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


for (B, H, T, D) in [(8, 16, 1024, 64), (4, 16, 2048, 64), (4, 8, 1024, 128), (2, 16, 4096, 128)]:
    q, k, v = (torch.randn(B, H, T, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    do = torch.randn(B, H, T, D, device="cuda", dtype=torch.bfloat16)
    flops_f = 4 * B * H * T * T * D / 2  # causal
    res = {"shape": [B, H, T, D]}
    for name, f in (("ours", lambda: flash_attention(q, k, v, causal=True)),
                    ("sdpa", lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True))):
        with torch.no_grad():
            tf = bench(f)
        def fb():
            o = f()
            torch.autograd.grad(o, (q, k, v), do)
        tfb = bench(fb)
        res[name] = {"fwd_ms": round(tf, 3), "fwd_tflops": round(flops_f / tf / 1e9, 1),
                     "fwd_bwd_ms": round(tfb, 3), "fwd_bwd_tflops": round(3.5 * flops_f / tfb / 1e9, 1)}
    print(json.dumps(res), flush=True)
