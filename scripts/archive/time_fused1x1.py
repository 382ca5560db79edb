"""Times the one-pass 1x1 backward against the separate dgrad(+BN prologue) and weight-gradient
passes on ResNet-50's first-stage 256 -> 64 1x1 conv at batch 512 (what ops/conv.py's timed choice
compares; profiles/conv1x1_bwd_fused_k512_attempts_1gpu.txt has the wider-conv attempts)."""
import json

import torch

from determined_amd import ops
from determined_amd.ops import conv as cv


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1000.0


def main():
    e = ops.ext()
    cl = torch.channels_last
    for n, hw, K, C in [(512, 56, 256, 64)]:
        yb = torch.randn(n, C, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        a, stats, _ = e.bn_act_fwd(yb, torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.2,
                                   None, None, 0.0, 1e-5, None, True, False, None)
        w = (torch.randn(K, C, 1, 1, device="cuda") / C ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
        dzn = torch.randn(n, K, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        yn = torch.randn_like(dzn)
        coef = torch.randn(3, K, device="cuda").contiguous()
        wt = cv._flip_weight(w)
        pro = [c for c in range(e.conv_num_cfgs()) if e.conv_pro_supported(dzn, wt, c)]
        t_fused = t(lambda: e.conv1x1_bwd_fused(dzn, yn, coef, w, a, yb, stats))
        t_d = {c: t(lambda c=c: e.conv_dgrad_bn(dzn, wt, 0, c, None, yb, None, stats, yn, coef)) for c in pro}
        gz = e.conv_dgrad_bn(dzn, wt, 0, pro[-1], None, yb, None, stats, yn, coef)[2]
        t_w = t(lambda: cv._wgrad(gz, a, w, 1, 0))
        hbm = (2 * n * hw * hw * K + 3 * n * hw * hw * C) * 2 / 1e9
        print(json.dumps({"shape": [n, hw, K, C], "fused_us": round(t_fused, 1),
                          "dgrad_pro_us": {str(c): round(v, 1) for c, v in t_d.items()}, "wgrad_us": round(t_w, 1),
                          "fused_min_bytes_gb": round(hbm, 3),
                          "fused_tb_s": round(hbm / (t_fused * 1e-6) / 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
