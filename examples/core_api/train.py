"""Core API example: a plain PyTorch training loop made cluster-aware step by step (reference:
``examples/tutorials/core_api/{0_start..4_distributed}.py``, which increment an integer; this one
trains a small regression MLP so the numbers mean something).

What each piece adds:
* metrics      -- ``core_context.train.report_training_metrics / report_validation_metrics``
* checkpoints  -- ``core_context.checkpoint.store_path`` / ``restore_path`` + ``info.latest_checkpoint``,
                  and ``core_context.preempt.should_preempt()`` to stop cleanly
* hp search    -- ``core_context.searcher.operations()`` drives the length; hyperparameters come
                  from ``info.trial.hparams``; ``op.report_completed(metric)`` closes the op
* distributed  -- ``DistributedContext.from_torch_distributed()`` under the torch_distributed
                  launcher; gradients are averaged by the RCCL bucket engine (parallel/ddp.py)

Run locally (``python train.py``) or on a cluster with ``det e create <yaml> .``.
"""

import logging
import os
import pathlib

import torch
import torch.distributed as dist
from torch import nn

import determined_amd as det
from determined_amd import core
from determined_amd.parallel.ddp import DistributedDataParallel


def make_data(n: int, seed: int):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 16, generator=g)
    w = torch.linspace(-1, 1, 16)
    return x, (x @ w).unsqueeze(1) + 0.05 * torch.randn(n, 1, generator=g)


def main(core_context: core.Context, hparams: dict, latest_checkpoint) -> None:
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    rank, size = core_context.distributed.rank, core_context.distributed.size
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(16, hparams["width"]), nn.GELU(), nn.Linear(hparams["width"], 1)).to(dev)
    ddp = DistributedDataParallel(model) if size > 1 else None
    opt = torch.optim.SGD(model.parameters(), lr=hparams["lr"], momentum=0.9)
    steps_done = 0
    if latest_checkpoint is not None:
        with core_context.checkpoint.restore_path(latest_checkpoint) as path:
            st = torch.load(pathlib.Path(path) / "state.pt", weights_only=True)
            model.load_state_dict(st["model"])
            opt.load_state_dict(st["opt"])
            steps_done = int(st["steps"])
    x, y = make_data(4096, 1)
    xv, yv = make_data(512, 2)
    bs = hparams["batch_size"]
    for op in core_context.searcher.operations():
        while steps_done < op.length:
            lo = ((steps_done * size + rank) * bs) % (len(x) - bs)
            xb, yb = x[lo:lo + bs].to(dev), y[lo:lo + bs].to(dev)
            loss = nn.functional.mse_loss((ddp or model)(xb), yb)
            opt.zero_grad(set_to_none=False)
            loss.backward()
            if ddp is not None:
                ddp.finish()
            opt.step()
            steps_done += 1
            if steps_done % 50 == 0 and rank == 0:
                core_context.train.report_training_metrics(steps_done, {"loss": float(loss)})
                op.report_progress(steps_done)
            if steps_done % 100 == 0 or steps_done == op.length:
                with torch.no_grad():
                    vloss = float(nn.functional.mse_loss(model(xv.to(dev)), yv.to(dev)))
                if rank == 0:
                    core_context.train.report_validation_metrics(steps_done, {"validation_loss": vloss})
                if rank == 0:  # replicas are identical: the chief writes the (unsharded) checkpoint
                    with core_context.checkpoint.store_path({"steps_completed": steps_done}) as (path, _uuid):
                        torch.save({"model": model.state_dict(), "opt": opt.state_dict(), "steps": steps_done},
                                   path / "state.pt")
                if core_context.preempt.should_preempt():
                    return
        if rank == 0:
            op.report_completed(vloss)


if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO)
    info = det.get_cluster_info()
    distributed = None
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
        distributed = core.DistributedContext.from_torch_distributed()
    if info is not None and info.task_type == "TRIAL":
        hp = info.trial.hparams
        latest = info.latest_checkpoint
        with core.init(distributed=distributed) as ctx:
            main(ctx, hp, latest)
    else:  # local run: a single op of 300 steps, checkpoints under ./checkpoints
        hp = {"lr": 0.05, "width": 64, "batch_size": 32}
        with core.init(distributed=distributed, checkpoint_storage=os.path.abspath("checkpoints")) as ctx:
            main(ctx, hp, None)
