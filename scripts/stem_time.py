#!/usr/bin/env python3
"""Time the ResNet stem (conv7x7/s2 -> BN -> ReLU -> maxpool) at the bench shape: the fused
stem_pool op (ops/conv.py stem_bn_pool) vs the separate stem-conv + BN/ReLU/max-pool kernels."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import determined_amd.ops as ops  # noqa: E402
from determined_amd.ops.conv import _StemPoolFn, stem_conv2d  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1024)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()

torch.manual_seed(0)
dev = torch.device("cuda", 0)
conv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(dev).to(torch.bfloat16)
bn = ops.BatchNormAct2d(64).to(dev).to(torch.bfloat16)
pool = torch.nn.MaxPool2d(3, 2, 1)
x = torch.randn(a.batch, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
g = torch.randn(a.batch, 64, 56, 56, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def fused():
    rm, rv, mom = bn.train_step_args()
    return _StemPoolFn.apply(x, conv.weight, bn.weight, bn.bias, rm, rv, mom, bn.eps, False)


def unfused():
    y, part = stem_conv2d(conv, x, with_stats=True)
    return bn.forward_maxpool(y, pool, stats_part=part)


def timeit(fn, backward):
    for _ in range(3):
        y = fn()
        if backward:
            y.backward(g)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        y = fn()
        if backward:
            y.backward(g)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / a.iters * 1e3


out = {}
for name, fn in (("fused", fused), ("unfused", unfused)):
    fwd = timeit(fn, False)
    both = timeit(fn, True)
    out[name] = {"fwd_us": round(fwd, 1), "bwd_us": round(both - fwd, 1), "total_us": round(both, 1)}
print(json.dumps({"batch": a.batch, **out}))
