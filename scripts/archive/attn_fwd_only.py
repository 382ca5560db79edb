#!/usr/bin/env python3
"""A few attention forward (+ optional backward) launches at the GPT-2 345M shape, for rocprofv3 PMC passes."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from determined_amd.ops.attention import flash_attention  # noqa: E402

bwd = len(sys.argv) > 1 and sys.argv[1] == "bwd"
B, H, T, D = 8, 16, 1024, 64
q, k, v = (torch.randn(B, H, T, D, device="cuda", dtype=torch.bfloat16, requires_grad=bwd) for _ in range(3))
do = torch.randn(B, H, T, D, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    o = flash_attention(q, k, v, causal=True)
    if bwd:
        torch.autograd.grad(o, (q, k, v), do)
torch.cuda.synchronize()
print("done")
