"""A/B: ResNet-50 (b512) 1x1 stride-1 convolution forward on MIOpen vs one hipBLASLt GEMM
(Y = X @ W^T on the channels-last [N*H*W, C] view)."""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
os.environ.setdefault("MIOPEN_USER_DB_PATH", os.path.join(ROOT, "determined_amd", "benchmarks", "miopen_db"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from conv1x1_gemm_ab import SHAPES, timed  # noqa: E402


def main():
    torch.backends.cudnn.benchmark = True
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    tot = {"miopen_fwd": 0.0, "gemm_fwd": 0.0}
    for hw, cin, cout in SHAPES:
        x = torch.randn(n, cin, hw, hw, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(cout, cin, 1, 1, device="cuda", dtype=torch.bfloat16) * 0.05
        x2, w2 = x.permute(0, 2, 3, 1).reshape(-1, cin), w.view(cout, cin)
        ref = F.conv2d(x, w)
        g = (x2 @ w2.t()).view(n, hw, hw, cout).permute(0, 3, 1, 2)
        r = {"hw": hw, "cin": cin, "cout": cout, "miopen_fwd": timed(lambda: F.conv2d(x, w)),
             "gemm_fwd": timed(lambda: x2 @ w2.t()),
             "rel_err": ((g.float() - ref.float()).abs().max() / ref.float().abs().max()).item()}
        for k in tot:
            tot[k] += r[k]
        print(json.dumps({k: (round(v, 1) if k in tot else v) for k, v in r.items()}), flush=True)
    print(json.dumps({"batch": n, "sum_us_per_shape_once": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
