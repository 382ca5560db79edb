#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 PyTorchTrial training throughput (samples/s, whole job).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it is launched
by ``torch.distributed.run`` (one rank per GPU, RCCL).  W untimed warmup steps, then EXACTLY
K timed steps bracketed by barrier + ``torch.cuda.synchronize()``; the max time over ranks is
used and rank 0 prints ONE JSON line.

The timed step is the full PyTorchTrial training step as run by
``determined_amd.pytorch`` (``examples/resnet50/model_def.py:ResNet50Trial.train_batch``):
bf16 channels-last forward/backward, bucketed RCCL all-reduce overlapped with backward,
fused multi-tensor SGD (momentum, weight decay, fp32 master weights) -- no work skipped.
Data: synthetic ImageNet-shaped batches (3x224x224, 1000 classes), random-init weights.
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# MIOpen find-db of the ResNet-50 convolutions measured on MI355X (written by MIOpen itself when
# torch.backends.cudnn.benchmark searches): a fresh box reuses it instead of re-searching every
# conv solver on every rank during warm-up.
_MIOPEN_DB = os.path.join(ROOT, "determined_amd", "benchmarks", "miopen_db")
if int(os.environ.get("WORLD_SIZE", "1")) > 1 and "MIOPEN_USER_DB_PATH" not in os.environ:
    # one private copy per rank: N processes never write the same find-db files concurrently
    import shutil
    import tempfile

    _priv = os.path.join(tempfile.gettempdir(), f"damd_miopen_db_rank{os.environ.get('LOCAL_RANK', '0')}_{os.getpid()}")
    shutil.copytree(_MIOPEN_DB, _priv, dirs_exist_ok=True)
    _MIOPEN_DB = _priv
os.environ.setdefault("MIOPEN_USER_DB_PATH", _MIOPEN_DB)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BASELINE = None  # BASELINE.json "published" is empty -> vs_baseline null


def parse() -> argparse.Namespace:
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=10)
    # 2048 images per GPU (78.5 GiB peak of the 288 GB HBM3E): one box, MIOpen immediate mode,
    # 1024 -> 14,945, 1536 -> 15,532, 2048 -> 15,679 samples/s (profiles/resnet50_batch_sweep_immediate_1gpu.txt;
    # earlier: 256 -> 12,526, 512 -> 14,050); the larger pixel count fills the 14x14 / 7x7 layers'
    # tiles across the 256 CUs
    p.add_argument("--batch", type=int, default=2048, help="per-GPU batch size")
    p.add_argument("--variant", default="bf16_master", choices=["bf16_master", "amp", "bf16_fp32bn"])
    p.add_argument("--no-harness", action="store_true", help="bypass the PyTorchTrial controller")
    p.add_argument("--bucket-mb", type=float, default=16.0)
    p.add_argument("--profile-steps", type=int, default=0)
    p.add_argument("--save-tune-db", default="", help="write the per-layer conv kernel choices after warm-up")
    p.add_argument("--no-pretune", action="store_true",
                   help="pick conv kernels inside the first warm-up step instead of a separate no-sync pass")
    # MIOpen immediate mode takes the solvers recorded in the in-tree find-db (searched once on an
    # MI355X, scripts/archive/gpu_finddb.sh) without re-running the search on every fresh box: batch 2048
    # starts in ~11 s instead of ~300 s at the same throughput (15,957 / 15,980 vs 15,910 / 15,957
    # samples/s, profiles/resnet50_b2048_finddb_vs_immediate_1gpu.txt)
    p.add_argument("--conv-benchmark", type=int, default=0,
                   help="1: let MIOpen search for the fastest conv solvers (torch.backends.cudnn.benchmark)")
    return p.parse_args()


def main() -> int:
    a = parse()
    # stdout carries exactly one line (rank 0's JSON): everything else written to fd 1 during the
    # run -- e.g. gloo's "[Gloo] Rank i is connected to ..." lines, printed by every rank when the
    # harness builds its gloo side groups -- goes to stderr
    sys.stdout.flush()
    stdout_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # one rank per GPU; the modulo and DAMD_BENCH_BACKEND=gloo only matter for rehearsing the
    # multi-rank path with several ranks on one GPU (RCCL refuses two ranks on one device)
    dev = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    torch.backends.cudnn.benchmark = bool(a.conv_benchmark)
    if world > 1:
        backend = os.environ.get("DAMD_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)

    from determined_amd.benchmarks.resnet50 import build_step

    step_fn, state = build_step(batch=a.batch, variant=a.variant, bucket_mb=a.bucket_mb,
                                use_harness=not a.no_harness)

    t_w = time.perf_counter()
    # kernel tuning and the first warm-up step may spend minutes in per-layer kernel timing and
    # MIOpen's solver search for shapes missing from the find-db: keep a heartbeat on stderr from
    # the start so supervisors do not mistake it for a hang
    import threading

    warm_done = threading.Event()

    def heartbeat() -> None:
        while not warm_done.wait(30.0):
            print(f"[bench] warming up ({time.perf_counter() - t_w:.0f}s)", file=sys.stderr, flush=True)

    if rank == 0:
        threading.Thread(target=heartbeat, daemon=True).start()
    if "tune" in state and not a.no_pretune:  # kernel choices outside the gradient all-reduce (all ranks alike)
        state["tune"]()
        if rank == 0:
            from determined_amd.ops.conv import tuning_seconds

            print(f"[bench] conv kernels tuned ({time.perf_counter() - t_w:.1f}s; {tuning_seconds():.1f}s timing "
                  f"candidates)", file=sys.stderr, flush=True)
    for i in range(a.warmup):
        step_fn()
        if rank == 0:  # progress on stderr (stdout carries only the JSON line)
            torch.cuda.synchronize()
            print(f"[bench] warmup {i + 1}/{a.warmup} {time.perf_counter() - t_w:.1f}s", file=sys.stderr, flush=True)
    warm_done.set()
    torch.cuda.synchronize()
    import determined_amd.ops as damd_ops

    damd_ops.conv_health_check()  # a stream-K hand-off time-out fails the run loudly
    if a.save_tune_db and rank == 0:
        from determined_amd.ops.conv import save_tune_db

        print(f"[bench] saved {save_tune_db(a.save_tune_db)} conv choices to {a.save_tune_db}", file=sys.stderr)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step_fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    damd_ops.conv_health_check()
    if rank == 0:
        print(f"[bench] peak GPU memory {torch.cuda.max_memory_allocated() / 2**30:.1f} GiB", file=sys.stderr, flush=True)
    loss = float(state["last_loss"]()) if "last_loss" in state else float("nan")
    if rank == 0 and os.environ.get("DAMD_TUNE_DUMP"):  # per-layer kernel choices (A/B analysis)
        from determined_amd.ops.conv import tuned_choices

        with open(os.environ["DAMD_TUNE_DUMP"], "a") as f:
            f.write(f"# DAMD_CONV_EXCLUDE={os.environ.get('DAMD_CONV_EXCLUDE', '')}\n")
            for k, v in sorted(tuned_choices().items(), key=str):
                f.write(f"{k} -> {v}\n")
    samples = a.batch * world * a.steps
    value = samples / dt
    if rank == 0:
        out = {
            "metric": "samples/sec (whole node) + scaling eff at 1/2/4/8 MI355X, PyTorchTrial ResNet-50",
            "value": round(value, 2),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1000, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (value / BASELINE) if BASELINE else None,
            "dtype": "bf16",
            "data": "synthetic (ImageNet-shaped 3x224x224, 1000 classes; random-init weights)",
            "config": {
                "model": "resnet50",
                "global_batch": a.batch * world,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "per_gpu_batch": a.batch,
                "variant": a.variant,
                "harness": not a.no_harness,
                "final_loss": round(loss, 4),
            },
        }
        sys.stdout.flush()
        os.dup2(stdout_fd, 1)
        print(json.dumps(out), flush=True)
        os.dup2(2, 1)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
