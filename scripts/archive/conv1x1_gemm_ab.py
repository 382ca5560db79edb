"""A/B: ResNet-50 (b512) 1x1 stride-1 convolution backward on MIOpen vs plain hipBLASLt GEMMs.

Channels-last activations are [M, C] row-major matrices, so dX = dY @ W and dW = dY^T @ X.
MIOpen's chosen solvers zero-fill their outputs before the CK/igemm kernels (see
profiles/resnet50_b512_1gpu_steady_state_r2.txt); this measures whether GEMMs beat them."""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(ROOT, "determined_amd", "benchmarks", "miopen_db"))

import torch  # noqa: E402

SHAPES = [(56, 64, 64), (56, 256, 64), (56, 64, 256), (28, 256, 128), (28, 512, 128), (28, 128, 512),
          (14, 512, 256), (14, 1024, 256), (14, 256, 1024), (7, 1024, 512), (7, 2048, 512), (7, 512, 2048)]


def timed(fn, it=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1000.0  # us


def main():
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    tot = {"miopen_dx": 0.0, "gemm_dx": 0.0, "miopen_dw": 0.0, "gemm_dw": 0.0}
    for hw, cin, cout in SHAPES:
        x = torch.randn(n, cin, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(n, cout, hw, hw, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(cout, cin, 1, 1, device=dev, dtype=torch.bfloat16) * 0.05
        args = (dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1)
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
        x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
        w2 = w.view(cout, cin)
        ref_dx = torch.ops.aten.convolution_backward(*args, [True, False, False])[0]
        ref_dw = torch.ops.aten.convolution_backward(*args, [False, True, False])[1]
        g_dx = (dy2 @ w2).view(n, hw, hw, cin).permute(0, 3, 1, 2)
        g_dw = (dy2.t() @ x2).view(cout, cin, 1, 1)
        err_dx = ((g_dx.float() - ref_dx.float()).abs().max() / ref_dx.float().abs().max()).item()
        err_dw = ((g_dw.float() - ref_dw.float()).abs().max() / ref_dw.float().abs().max()).item()
        r = {
            "hw": hw, "cin": cin, "cout": cout,
            "miopen_dx": timed(lambda: torch.ops.aten.convolution_backward(*args, [True, False, False])),
            "gemm_dx": timed(lambda: dy2 @ w2),
            "miopen_dw": timed(lambda: torch.ops.aten.convolution_backward(*args, [False, True, False])),
            "gemm_dw": timed(lambda: dy2.t() @ x2),
            "rel_err_dx": err_dx, "rel_err_dw": err_dw,
        }
        for k in tot:
            tot[k] += r[k]
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) and k[0] != "r" else v) for k, v in r.items()}),
              flush=True)
        del x, dy, ref_dx, ref_dw, g_dx, g_dw
    print(json.dumps({"batch": n, "sum_us_per_shape_once": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
