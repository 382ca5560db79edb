#!/usr/bin/env python3
"""Per-shape timing of ResNet-50 convolutions (bf16, NHWC, batch 256): MIOpen vs GEMM formulation."""
import json
import sys

import torch
import torch.nn.functional as F

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
bench_mode = int(sys.argv[2]) if len(sys.argv) > 2 else 0
torch.backends.cudnn.benchmark = bool(bench_mode)
dev = "cuda"

# (cin, cout, k, stride, H_in, count in network)
SHAPES = [
    (3, 64, 7, 2, 224, 1),
    (64, 64, 1, 1, 56, 1), (64, 64, 3, 1, 56, 3), (64, 256, 1, 1, 56, 4), (256, 64, 1, 1, 56, 2),
    (256, 128, 1, 1, 56, 1), (128, 128, 3, 2, 56, 1), (128, 512, 1, 1, 28, 4), (256, 512, 1, 2, 56, 1),
    (512, 128, 1, 1, 28, 3), (128, 128, 3, 1, 28, 3),
    (512, 256, 1, 1, 28, 1), (256, 256, 3, 2, 28, 1), (256, 1024, 1, 1, 14, 6), (512, 1024, 1, 2, 28, 1),
    (1024, 256, 1, 1, 14, 5), (256, 256, 3, 1, 14, 5),
    (1024, 512, 1, 1, 14, 1), (512, 512, 3, 2, 14, 1), (512, 2048, 1, 1, 7, 3), (1024, 2048, 1, 2, 14, 1),
    (2048, 512, 1, 1, 7, 2), (512, 512, 3, 1, 7, 2),
]


def timeit(fn, iters=10):
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


tot_conv, tot_gemm = 0.0, 0.0
rows = []
for cin, cout, k, st, H, cnt in SHAPES:
    x = torch.randn(B, cin, H, H, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    w.requires_grad_(True)
    pad = k // 2
    y = F.conv2d(x, w, stride=st, padding=pad)
    gy = torch.randn_like(y)

    def conv_fb():
        out = F.conv2d(x, w, stride=st, padding=pad)
        gx, gw = torch.autograd.grad(out, (x, w), gy)

    t_conv = timeit(conv_fb)
    t_fwd = timeit(lambda: F.conv2d(x, w, stride=st, padding=pad))
    t_gemm = None
    if k == 1:
        xs = x[:, :, ::st, ::st] if st > 1 else x
        Ho = xs.shape[2]
        xm = xs.permute(0, 2, 3, 1).reshape(-1, cin).contiguous() if st > 1 else x.permute(0, 2, 3, 1).reshape(-1, cin)
        wm = w.reshape(cout, cin)
        gym = gy.permute(0, 2, 3, 1).reshape(-1, cout)

        def gemm_fb():
            out = xm @ wm.t()
            gx = gym @ wm
            gw = gym.t() @ xm

        t_gemm = timeit(gemm_fb)
    tot_conv += t_conv * cnt
    tot_gemm += (t_gemm if t_gemm is not None else t_conv) * cnt
    flops = 2 * B * (H // st) ** 2 * cin * cout * k * k * 3
    rows.append(dict(shape=(cin, cout, k, st, H), cnt=cnt, conv_ms=round(t_conv, 4), fwd_ms=round(t_fwd, 4),
                     gemm_ms=None if t_gemm is None else round(t_gemm, 4),
                     conv_tflops=round(flops / t_conv / 1e9, 1)))
    print(json.dumps(rows[-1]), flush=True)
print(json.dumps({"bench_mode": bench_mode, "total_conv_ms": round(tot_conv, 3), "total_best_gemm_ms": round(tot_gemm, 3)}))
