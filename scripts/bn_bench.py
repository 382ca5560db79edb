#!/usr/bin/env python3
"""BN+act kernel bandwidth on the ResNet-50 shapes at batch 512 (bf16 NHWC): forward (stats +
apply) and backward (reduce + apply) of ``csrc/bn.hip`` in GB/s of compulsory HBM traffic."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from determined_amd import ops  # noqa: E402

e = ops.ext()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
SHAPES = [(112, 64, False), (56, 64, False), (56, 256, True), (28, 128, False), (28, 512, True),
          (14, 256, False), (14, 1024, True), (7, 512, False), (7, 2048, True)]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    t.record()
    torch.cuda.synchronize()
    return s.elapsed_time(t) / iters


tot = {"fwd": 0.0, "bwd": 0.0}
for H, C, res in SHAPES:
    x = torch.randn(B, C, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x) if res else None
    w = torch.ones(C, device="cuda", dtype=torch.bfloat16)
    b = torch.zeros(C, device="cuda", dtype=torch.bfloat16)
    rm = torch.zeros(C, device="cuda")
    rv = torch.ones(C, device="cuda")
    y, stats, mask = e.bn_act_fwd(x, w, b, rm, rv, 0.1, 1e-5, r, True, True)
    dy = torch.randn_like(x)
    nbytes = x.numel() * 2
    tf = timeit(lambda: e.bn_act_fwd(x, w, b, rm, rv, 0.1, 1e-5, r, True, True))
    tb = timeit(lambda: e.bn_act_bwd(dy, x, None if res else None, stats, w, True, res, mask if res else None, None))
    # compulsory passes: fwd = stats(1R) + apply(1R [+1R res] + 1W); bwd = reduce(2R) + apply(2R + 1W [+1W dres])
    pf = 3 + (1 if res else 0)
    pb = 5 + (1 if res else 0)
    tot["fwd"] += tf
    tot["bwd"] += tb
    print(json.dumps({"shape": [B, H, H, C], "res": res, "fwd_ms": round(tf, 4), "bwd_ms": round(tb, 4),
                      "fwd_GBps": round(pf * nbytes / tf / 1e6), "bwd_GBps": round(pb * nbytes / tb / 1e6)}),
          flush=True)
print(json.dumps({k: round(v, 3) for k, v in tot.items()}))
# ceiling references on the same box: device copy (1R + 1W) and an elementwise add (2R + 1W)
big = torch.randn(512 * 56 * 56 * 256, device="cuda", dtype=torch.bfloat16)
big2 = torch.randn_like(big)
out = torch.empty_like(big)
tc = timeit(lambda: out.copy_(big))
ta = timeit(lambda: torch.add(big, big2, out=out))
nb = big.numel() * 2
print(json.dumps({"copy_GBps": round(2 * nb / tc / 1e6), "add_GBps": round(3 * nb / ta / 1e6)}))
