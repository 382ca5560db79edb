#!/usr/bin/env python3
"""Per-config timing of the ResNet-50 3x3 stride-1 layers at the bench batch: every conv config that
serves the layer (conv_igemm.hip generic / halo, conv3x3v2.hip padded-halo) for the forward with BN
statistics, the BN+ReLU-prologue forward, the input gradient with the BN-backward epilogue, and the
same with the deferred BN-backward apply prologue, and the weight gradient.  One JSON line per (layer, pass,
config).

    python scripts/v2_bench.py [--batch 2048] [--out gpurun_out/v2_bench.jsonl]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("DAMD_AB_ROOT", ROOT))  # A/B: another build of the package
import torch  # noqa: E402

CL = torch.channels_last


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / reps * 1000.0)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--out", default="gpurun_out/v2_bench.jsonl")
    ap.add_argument("--layers", default="64x56,128x28,256x14")
    ap.add_argument("--passes", default="fwd_stats,fwd_bnrelu_pro,dgrad_bn_epi,dgrad_bn_epi_pro2,wgrad")
    a = ap.parse_args()
    from determined_amd import ops

    e = ops.ext()
    nv2 = e.conv_v2_num_cfgs()
    base = e.conv_num_cfgs() - nv2
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    out = open(a.out, "w")
    for spec in a.layers.split(","):
        c, hw = (int(v) for v in spec.split("x"))
        n = a.batch
        torch.manual_seed(0)
        x = torch.randn(n, c, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(c, c, 3, 3, device="cuda") / (9 * c) ** 0.5).to(torch.bfloat16).contiguous(memory_format=CL)
        wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=CL)
        a_, stats, _ = e.bn_act_fwd(x, torch.rand(c, device="cuda") + 0.5, torch.randn(c, device="cuda") * 0.2,
                                    None, None, 0.0, 1e-5, None, True, False, None)
        yn = torch.randn_like(x)
        coef = torch.randn(3, c, device="cuda").contiguous()
        flops = 2.0 * n * hw * hw * c * c * 9
        cfgs = [k for k in range(e.conv_num_cfgs()) if e.conv_supported(x, w, k, 1, 1)]
        passes = {
            "fwd_stats": lambda k: e.conv_fwd(x, w, 1, 1, True, k, 0),
            "fwd_bnrelu_pro": (lambda k: e.conv_bnact_fwd(x, w, None, stats, False, k, None))
            if True else None,
            "dgrad_bn_epi": lambda k: e.conv_dgrad_bn(x, wt, 1, k, None, x, None, stats, None, None),
            "dgrad_bn_epi_pro2": lambda k: e.conv_dgrad_bn(x, wt, 1, k, None, x, None, stats, yn, coef),
        }
        for pname, fn in passes.items():
            if pname not in a.passes.split(","):
                continue
            for k in cfgs:
                if pname in ("fwd_bnrelu_pro", "dgrad_bn_epi_pro2") and not e.conv_pro_supported(x, w, k):
                    continue
                try:
                    us = timeit(lambda: fn(k))
                except RuntimeError as err:
                    print(f"{spec} {pname} cfg {k}: {err}", flush=True)
                    continue
                rec = {"layer": spec, "batch": n, "pass": pname, "cfg": k, "v2": k >= base, "us": round(us, 1),
                       "tflops": round(flops / us / 1e6, 1)}
                out.write(json.dumps(rec) + "\n")
                out.flush()
                print(json.dumps(rec), flush=True)
        # weight gradient: conv_igemm.hip's split-pixel configs, the 3x3 halo kernels ("h<cfg>": h0 / h1
        # conv_igemm.hip, h2.. conv3x3v2.hip) and MIOpen
        dyw = yn
        wg = {f"w{k}": (lambda k=k: e.conv_wgrad(x, dyw, w, 1, 1, k, 0))
              for k in range(e.wgrad_num_cfgs()) if e.wgrad_supported(x, dyw, w.shape[0], k)}
        wg.update({f"h{k}": (lambda k=k: e.conv3x3_wgrad(x, dyw, w, k, 0))
                   for k in range(e.wgrad3x3_num_cfgs()) if e.wgrad3x3_supported(x, dyw, w, k)})
        wg["miopen"] = lambda: torch.ops.aten.convolution_backward(dyw, x, w, None, [1, 1], [1, 1], [1, 1], False,
                                                                   [0, 0], 1, [False, True, False])[1]
        for k, fn in (wg.items() if "wgrad" in a.passes.split(",") else ()):
            try:
                us = timeit(fn)
            except RuntimeError as err:
                print(f"{spec} wgrad {k}: {err}", flush=True)
                continue
            v2 = k.startswith("h") and int(k[1:]) >= 2
            rec = {"layer": spec, "batch": n, "pass": "wgrad", "cfg": k, "v2": v2, "us": round(us, 1),
                   "tflops": round(flops / us / 1e6, 1)}
            out.write(json.dumps(rec) + "\n")
            out.flush()
            print(json.dumps(rec), flush=True)
        del x, w, wt, a_, yn
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
