"""GPT-2 ZeRO benchmark (BASELINE config "GPT-2 345M DeepSpeedTrial ZeRO-2").

``python -m determined_amd.benchmarks.gpt2 [--model gpt2-medium] [--mb 8] [--seq 1024]
[--stage 2] [--steps 20] [--warmup 5]`` (under torchrun for N GPUs).  Runs the real ZeRO
engine step (forward, backward with bucketed reduce-scatter, fused AdamW on the shard with
clipping, all-gather) on GPU-resident synthetic token batches; prints one JSON line with
whole-job tokens/s and samples/s.  bf16 weights/activations, fp32 master + moments.
"""

import argparse
import json
import os
import time

import torch
import torch.distributed as dist


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--mb", type=int, default=8)
    ap.add_argument("--gas", type=int, default=1)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--stage", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--ckpt", action="store_true", help="activation checkpointing")
    ap.add_argument("--bucket", type=int, default=16 * 1024 * 1024)
    default_tun = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunableop", "gpt2_345m_mb8.csv")
    # in-tree TunableOp choices (+1% same-box at mb 8; shapes not in the file keep hipBLASLt's
    # default); --tunable "" disables
    ap.add_argument("--tunable", default=default_tun if os.path.exists(default_tun) else "",
                    help="PyTorch TunableOp GEMM results file (use it)")
    ap.add_argument("--tune", action="store_true", help="with --tunable: search and (re)write the file")
    a = ap.parse_args()
    if a.tunable:
        # hipBLASLt/rocBLAS solution choice per GEMM shape from a results file; --tune searches
        # during warm-up (bounded per solution) and writes the file at the end
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(a.tune)
        torch.cuda.tunable.set_max_tuning_duration(20)
        torch.cuda.tunable.set_max_tuning_iterations(20)
        torch.cuda.tunable.set_filename(a.tunable)
        if not a.tune:
            torch.cuda.tunable.read_file(a.tunable)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("nccl", device_id=dev)
    from determined_amd.models.gpt2 import gpt2
    from determined_amd.parallel import zero

    torch.manual_seed(0)
    model = gpt2(a.model, dropout=a.dropout, activation_checkpointing=a.ckpt)
    n_params = model.num_parameters()
    decay = [p for n, p in model.named_parameters() if p.ndim >= 2]
    no_decay = [p for n, p in model.named_parameters() if p.ndim < 2]
    cfg = {
        "train_micro_batch_size_per_gpu": a.mb, "gradient_accumulation_steps": a.gas,
        "bf16": {"enabled": True}, "gradient_clipping": 1.0,
        "optimizer": {"type": "AdamW", "params": {"lr": 1.5e-4, "betas": [0.9, 0.95], "weight_decay": 0.1}},
        "scheduler": {"type": "WarmupDecayLR", "params": {"warmup_max_lr": 1.5e-4, "warmup_num_steps": 100,
                                                          "total_num_steps": 10000, "warmup_type": "linear"}},
        "zero_optimization": {"stage": a.stage, "reduce_bucket_size": a.bucket},
    }
    engine, *_ = zero.initialize(model=model, config=cfg,
                                 model_parameters=[{"params": decay, "weight_decay": 0.1},
                                                   {"params": no_decay, "weight_decay": 0.0}])
    g = torch.Generator(device=dev).manual_seed(1 + local)
    vocab = model.config.vocab_size
    pool = [torch.randint(0, vocab, (a.mb, a.seq), device=dev, generator=g) for _ in range(2)]
    it = [0]

    def step() -> torch.Tensor:
        loss = None
        for _ in range(a.gas):
            x = pool[it[0] % 2]
            it[0] += 1
            loss = engine(x, labels=x)
            engine.backward(loss)
            engine.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t)
    samples = a.mb * a.gas * world * a.steps
    tokens = samples * a.seq
    # 6 * N * tokens (+ attention 12 * L * d * T per token) model FLOPs
    L, d = model.config.n_layer, model.config.n_embd
    flops_per_token = 6 * n_params + 12 * L * d * a.seq
    tflops = flops_per_token * tokens / dt / 1e12 / world
    if (dist.get_rank() if world > 1 else 0) == 0:
        print(json.dumps({
            "metric": "tokens/sec (whole job), GPT-2 ZeRO", "value": round(tokens / dt, 1), "unit": "tokens/s",
            "samples_per_sec": round(samples / dt, 2), "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(1000 * dt / a.steps, 2), "model_tflops_per_gpu": round(tflops, 1),
            "loss": round(float(loss), 4), "dtype": "bf16", "data": "synthetic",
            "config": {"model": a.model, "params": n_params, "micro_batch": a.mb, "gas": a.gas, "seq_len": a.seq,
                       "zero_stage": a.stage, "global_batch": a.mb * a.gas * world,
                       "activation_checkpointing": a.ckpt},
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
