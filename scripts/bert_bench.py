#!/usr/bin/env python3
"""BERT-base masked-LM training throughput on one GPU (BASELINE config #5's model and precision:
bf16 autocast as the HF Trainer runs it with ``--bf16``): the step the Trainer executes
(forward, loss, backward, optimizer step, zero_grad) timed in a plain loop so the number is not
diluted by the Trainer's logging.  Variants: ``fused`` (determined_amd.transformers.accelerate +
fused AdamW), ``fused_bf16w`` (the same with bf16 parameters and fp32 master weights in the fused AdamW:
no per-step autocast weight casts), ``fused_bf16w_graph`` (that step captured once into a hipGraph and
replayed: determined_amd.utils.graphs.GraphedStep) and ``stock`` (HF SDPA attention + torch fused AdamW).  One JSON line per variant.

    python scripts/bert_bench.py [--batch 64] [--seq 128] [--steps 30] [--warmup 10] [--variants fused,stock]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def build(variant: str, seq: int, dropout: float):
    import transformers

    from determined_amd.transformers import accelerate

    cfg = transformers.BertConfig(max_position_embeddings=max(512, seq), hidden_dropout_prob=dropout,
                                  attention_probs_dropout_prob=dropout, attn_implementation="sdpa")
    torch.manual_seed(0)
    model = transformers.BertForMaskedLM(cfg).cuda()
    if variant in ("fused", "fused_bf16w", "fused_bf16w_graph"):
        accelerate(model)
        from determined_amd.ops import FusedAdamW

        bf16w = variant != "fused"
        if bf16w:  # bf16 parameters, fp32 master weights in the optimizer
            model = model.to(torch.bfloat16)
        opt = FusedAdamW(model.parameters(), lr=1e-4, weight_decay=0.01, master_weights=bf16w)
    else:
        opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01, fused=True)
    return model, opt


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--variants", default="fused,fused_bf16w,fused_bf16w_graph,stock")
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    ids = torch.randint(1000, 30522, (a.batch, a.seq), device="cuda", generator=g)
    labels = torch.where(torch.rand(a.batch, a.seq, device="cuda", generator=g) < 0.15, ids, torch.full_like(ids, -100))
    mask = torch.ones_like(ids)
    for variant in a.variants.split(","):
        model, opt = build(variant, a.seq, a.dropout)
        model.train()

        graphed = variant.endswith("_graph")

        def step():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = model(input_ids=ids, attention_mask=mask, labels=labels).loss
            loss.backward()
            opt.step()
            opt.zero_grad(set_to_none=not graphed)  # a captured step keeps its gradient buffers
            return loss

        if graphed:  # the whole step as one hipGraph (determined_amd.utils.graphs)
            from determined_amd.utils.graphs import GraphedStep

            step = GraphedStep(step, warmup=3)
        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            loss = step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        print(json.dumps({"model": "bert-base-mlm", "variant": variant, "batch": a.batch, "seq_len": a.seq,
                          "dtype": "bf16-autocast", "dropout": a.dropout, "ms_per_step": round(dt * 1e3, 2),
                          "tokens_per_s": round(a.batch * a.seq / dt, 1), "loss": round(float(loss), 4)}), flush=True)
        del model, opt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
