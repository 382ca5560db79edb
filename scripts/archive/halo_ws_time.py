#!/usr/bin/env python3
"""3x3 halo conv configs (and the generic configs for comparison) at the bench
shapes (batch 1024): plain forward + BN statistics, the BN-apply prologue forward (PRO 1) and the
input gradient with the deferred BN-backward apply + BN-backward epilogue (PRO 2), per config."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from determined_amd import ops  # noqa: E402

e = ops.ext()
cl = torch.channels_last
B = int(os.environ.get("HALO_BATCH", "1024"))


def timeit(fn, reps=10):
    fn()
    ts = []
    for _ in range(5):
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(reps):
            fn()
        s1.record()
        s1.synchronize()
        ts.append(s0.elapsed_time(s1) * 1000.0 / reps)
    ts.sort()
    return round(ts[2], 1)


for c, hw, cfgs in ((64, 56, (7, 19, 26)), (128, 28, (6, 8, 18, 20, 27, 12, 22)), (256, 14, (6, 9, 21, 27, 28, 12, 22))):
    torch.manual_seed(0)
    x = torch.randn(B, c, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(c, c, 3, 3, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=cl)
    wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=cl)
    stats = torch.stack([torch.zeros(c), torch.ones(c), torch.rand(c) + 0.5, torch.randn(c) * 0.1]).cuda().contiguous()
    yn = torch.randn_like(x)
    coef = torch.randn(3, c, device="cuda").contiguous()
    ref = None
    for cfg in cfgs:
        if not e.conv_supported(x, w, cfg, 1, 1):
            continue
        row = {"c": c, "hw": hw, "cfg": cfg}
        y, _ = e.conv_fwd(x, w, 1, 1, True, cfg, 0)
        if ref is None:
            ref = y.float()
        row["err"] = float(((y.float() - ref).norm() / ref.norm()).item())
        row["fwd_stats_us"] = timeit(lambda: e.conv_fwd(x, w, 1, 1, True, cfg, 0))
        if e.conv_pro_supported(x, w, cfg):
            row["fwd_pro1_us"] = timeit(lambda: e.conv_bnact_fwd(x, w, None, stats, False, cfg, None))
            row["dgrad_pro2_bnb_us"] = timeit(lambda: e.conv_dgrad_bn(x, wt, 1, cfg, None, yn, None, stats, x, coef))
        print(json.dumps(row), flush=True)
