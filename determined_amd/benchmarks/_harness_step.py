"""Benchmark step through the real PyTorchTrial harness.

Builds ``examples/resnet50/model_def.py:ResNet50Trial`` under ``pytorch.init()`` and times the
controller's per-batch path (``_PyTorchTrialController._train_batch``: to_device, the trial's
``train_batch`` -> ``context.backward`` (bucketed RCCL all-reduce) -> ``context.step_optimizer``
(fused SGD), LR scheduler stepping, metric bookkeeping) plus the once-per-reporting-period
metric aggregation, exactly as ``Trainer.fit`` runs them.  Batches are synthetic ImageNet-shaped
tensors kept resident on the GPU.
"""

import importlib.util
import os
from typing import Any, Callable, Dict, Tuple

import torch

from determined_amd import pytorch
from determined_amd.pytorch._trial import Batch, _PyTorchTrialController

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _load_trial_cls():
    spec = importlib.util.spec_from_file_location("resnet50_model_def",
                                                  os.path.join(ROOT, "examples", "resnet50", "model_def.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # type: ignore[union-attr]
    return mod.ResNet50Trial


def harness_step(batch: int, variant: str, bucket_mb: float, device: torch.device
                 ) -> Tuple[Callable[[], None], Dict[str, Any]]:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    hparams = {"global_batch_size": batch * world, "lr": 0.1, "momentum": 0.9, "weight_decay": 5e-5,
               "dtype": "bf16" if variant != "fp32" else "fp32", "warmup_batches": 100, "total_batches": 10000}
    exp_conf = {"scheduling_unit": 100, "optimizations": {"average_training_metrics": True}, "data": {}}
    cm = pytorch.init(hparams=hparams, exp_conf=exp_conf, ddp_bucket_mb=bucket_mb)
    ctx = cm.__enter__()
    trial = _load_trial_cls()(ctx)
    ctrl = _PyTorchTrialController(
        trial_inst=trial, context=ctx, checkpoint_period=Batch(0), validation_period=Batch(0),
        reporting_period=Batch(100), smaller_is_better=True, steps_completed=0, latest_checkpoint=None,
        local_training=True, test_mode=False, searcher_metric_name="validation_loss", checkpoint_policy="none",
        step_zero_validation=False, max_length=Batch(10**9), global_batch_size=batch * world)
    ctx._epoch_len = 10**9
    g = torch.Generator(device=device)
    g.manual_seed(1234 + ctx.distributed.rank)
    pool = []
    for _ in range(2):
        x = torch.randn(batch, 3, 224, 224, generator=g, device=device, dtype=torch.float32)
        x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (batch,), generator=g, device=device)
        pool.append((x, y))
    state: Dict[str, Any] = {"i": 0, "metrics": [], "ctx_manager": cm, "ctx": ctx}

    def step() -> None:
        i = state["i"]
        ctx._current_batch_idx = i
        state["metrics"].append(ctrl._train_batch(pool[i % len(pool)], 0, i))
        ctrl.state.batches_trained += 1
        state["i"] = i + 1
        if len(state["metrics"]) == 100:  # reporting period: one aggregation + D2H per 100 batches
            state["last_report"] = ctrl._aggregate_training_metrics(state["metrics"])
            state["metrics"] = []

    def last_loss() -> float:
        if state["metrics"]:
            return float(state["metrics"][-1]["loss"].float().item())
        return float(state.get("last_report", {}).get("avg_metrics", {}).get("loss", float("nan")))

    def tune() -> None:
        """One forward/backward outside the gradient all-reduce (DDP no_sync, no optimizer step):
        every conv layer picks its kernels (ops/conv.py) while no RCCL traffic shares the GPU, so
        all ranks of a multi-GPU run time their candidates alike; gradients are dropped after."""
        import contextlib

        import torch.distributed as dist
        import torch.nn.functional as F

        from determined_amd.ops.conv import agree_across_ranks

        x, yl = pool[0]
        sync_off = ctx._ddp[0].no_sync() if ctx._ddp else contextlib.nullcontext()
        # multi-GPU: candidate timings averaged over the ranks (a gloo group), so every rank runs
        # the same kernels and no rank is slowed by a noisy pick
        group = dist.new_group(backend="gloo") if dist.is_initialized() and dist.get_world_size() > 1 else None
        with sync_off, agree_across_ranks(group):
            F.cross_entropy(trial.model(trial._prep(x)).float(), yl).backward()
        for m in ctx.models:
            m.zero_grad(set_to_none=True)
        torch.cuda.synchronize()

    state["last_loss"] = last_loss
    state["tune"] = tune
    return step, state
