"""Distributed batch inference over a dataset (reference:
``harness/determined/pytorch/experimental/_torch_batch_process.py``).

``torch_batch_process(MyProcessor, dataset, batch_size=...)`` shards ``dataset`` across every
slot (rank ``r`` gets batches ``r, r+N, ...``), calls ``MyProcessor.process_batch`` per batch,
checkpoints the number of completed batches every ``checkpoint_interval`` batches (minimum
over ranks, so a restarted task resumes without gaps), reports progress, honours preemption,
and reduces any wrapped ``MetricReducer`` across ranks at the end.  Outputs written through
``context.upload_path()`` land in ``<storage>/<output uuid>/rank_<r>`` (stable across
restarts of the same task).

MI355X-native additions: ``prepare_model_for_inference(model, dtype=torch.bfloat16,
channels_last=True)`` casts once for MFMA-friendly bf16 inference, and batches are moved to
the GPU with non-blocking copies from pinned memory.  Off-cluster the function also runs
(one local worker) so processors can be developed without a master.
"""

import abc
import contextlib
import json
import logging
import math
import os
import pathlib
import uuid
from typing import Any, ContextManager, Dict, Iterator, Optional, Type

import torch
from torch import nn

from determined_amd import core
from determined_amd._info import get_cluster_info
from determined_amd.pytorch import _data
from determined_amd.pytorch._reducer import _PyTorchReducerContext

logger = logging.getLogger("determined_amd.pytorch.experimental")

DEFAULT_BATCH_SIZE = 1


def get_default_device(core_context: Any) -> torch.device:
    if torch.cuda.is_available() and torch.cuda.device_count() > 0:
        return torch.device("cuda", core_context.distributed.local_rank % torch.cuda.device_count())
    return torch.device("cpu")


class TorchBatchProcessorContext(_PyTorchReducerContext):
    def __init__(self, core_context: Any, storage_path: str) -> None:
        super().__init__(core_context.distributed.allgather)
        self._core_context = core_context
        self._distributed = core_context.distributed
        self.device = get_default_device(core_context)
        self._storage_path = storage_path
        self._use_default_storage = False
        self._hparams: Optional[Dict[str, Any]] = None

    def get_hparams(self) -> Dict[str, Any]:
        if self._hparams is None:
            info = get_cluster_info()
            self._hparams = dict(info.trial.hparams) if info is not None and info.task_type == "TRIAL" else {}
        return self._hparams

    def to_device(self, data: Any) -> Any:
        return _data.to_device(data, self.device)

    def get_tensorboard_path(self) -> pathlib.Path:
        return self._core_context.train.get_tensorboard_path()

    def prepare_model_for_inference(self, model: nn.Module, dtype: Optional[torch.dtype] = None,
                                    channels_last: bool = False) -> nn.Module:
        model.eval()
        model.to(self.device)
        if dtype is not None:
            model.to(dtype)
        if channels_last:
            model.to(memory_format=torch.channels_last)
        return model

    def upload_path(self) -> ContextManager[pathlib.Path]:
        """Files written inside the context are stored under this rank's output directory."""
        self._use_default_storage = True
        return self._core_context.checkpoint._storage_manager.store_path(self._storage_path)

    def report_metrics(self, group: str, steps_completed: int, metrics: Dict[str, Any]) -> None:
        self._core_context.train.report_metrics(group=group, steps_completed=steps_completed, metrics=metrics)

    def report_task_using_checkpoint(self, checkpoint: Any) -> None:
        """Link this task to ``checkpoint``: the metrics it reports become the checkpoint's
        ``get_metrics()`` (core_context.experimental; chief only, like the reference)."""
        if self._distributed.get_rank() == 0:
            self._core_context.experimental.report_task_using_checkpoint(checkpoint)

    def report_task_using_model_version(self, model_version: Any) -> None:
        if self._distributed.get_rank() == 0:
            self._core_context.experimental.report_task_using_model_version(model_version)

    def get_distributed_rank(self) -> int:
        return self._distributed.get_rank()

    def get_distributed_size(self) -> int:
        return self._distributed.get_size()


class TorchBatchProcessor(metaclass=abc.ABCMeta):
    def __init__(self, context: TorchBatchProcessorContext) -> None:
        pass

    @abc.abstractmethod
    def process_batch(self, batch: Any, batch_idx: int) -> None:
        pass

    def on_checkpoint_start(self) -> None:  # noqa: B027 - optional hook
        """Flush buffered outputs before progress is checkpointed."""

    def on_finish(self) -> None:  # noqa: B027 - optional hook
        """Called once after the last batch on every rank."""


def _initialize_distributed_backend() -> Optional[core.DistributedContext]:
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return None
    import torch.distributed as dist

    if not dist.is_initialized():
        if torch.cuda.is_available():
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    return core.DistributedContext.from_torch_distributed()


def _checkpoint_progress(core_context: Any, steps_completed: int, output_uuid: str) -> None:
    """Record min(steps over ranks) as a checkpoint so a restart resumes without gaps."""
    steps = core_context.distributed.gather(steps_completed)
    if core_context.distributed.get_rank() == 0:
        done = min(steps) if steps else steps_completed
        with core_context.checkpoint.store_path({"steps_completed": done, "default_output_uuid": output_uuid}) as \
                (path, _):
            with open(os.path.join(path, "batch_completed.json"), "w") as f:
                json.dump({"batch_completed": done}, f)


def _reduce_metrics(ctx: TorchBatchProcessorContext, core_context: Any, steps_completed: int) -> Dict[str, Any]:
    wrapped = list(ctx._wrapped_reducers) if hasattr(ctx, "_wrapped_reducers") else []
    if not wrapped:
        return {}
    metrics = ctx.reduce_metrics(for_training=False)
    if core_context.distributed.get_rank() == 0 and metrics:
        core_context.train.report_validation_metrics(steps_completed=steps_completed, metrics=metrics)
    return metrics or {}


def _validate_dataloader_kwargs(kw: Dict[str, Any], batch_size: Optional[int]) -> None:
    if kw.get("shuffle"):
        raise ValueError("'shuffle' must be false for accurate sharding and checkpointing")
    for k in ("sampler", "batch_sampler"):
        if k in kw:
            raise ValueError(f"remove '{k}': torch_batch_process builds its own sharded sampler")
    if batch_size is not None and "batch_size" in kw:
        raise ValueError("batch_size is passed into torch_batch_process and dataloader_kwargs")


def torch_batch_process(batch_processor_cls: Type[TorchBatchProcessor], dataset: Any,
                        batch_size: Optional[int] = None, max_batches: Optional[int] = None,
                        checkpoint_interval: int = 5, dataloader_kwargs: Optional[Dict[str, Any]] = None,
                        distributed_context: Optional[core.DistributedContext] = None,
                        checkpoint_storage: Any = None) -> None:
    if checkpoint_interval <= 0:
        raise ValueError("checkpoint_interval should be a positive integer")
    kw = dict(dataloader_kwargs or {})
    _validate_dataloader_kwargs(kw, batch_size)
    if batch_size is None:
        batch_size = int(kw.pop("batch_size", DEFAULT_BATCH_SIZE))
    if not hasattr(dataset, "__len__"):
        raise TypeError("dataset must implement __len__()")
    dist_ctx = distributed_context or _initialize_distributed_backend()
    with core.init(distributed=dist_ctx, checkpoint_storage=checkpoint_storage) as core_context:
        rank = core_context.distributed.get_rank()
        workers = core_context.distributed.get_size()
        info = get_cluster_info()
        latest = info.latest_checkpoint if info is not None else None
        output_uuid = core_context.distributed.broadcast(str(uuid.uuid4()) if rank == 0 else None)
        skip = 0
        if latest is not None:
            with core_context.checkpoint.restore_path(latest) as p:
                md = json.loads((pathlib.Path(p) / "metadata.json").read_text())
            skip = int(md["steps_completed"])
            output_uuid = md.get("default_output_uuid", output_uuid)
            logger.info("resuming batch processing after %d batches", skip)
        ctx = TorchBatchProcessorContext(core_context, f"{output_uuid}/rank_{rank}")
        processor = batch_processor_cls(context=ctx)
        if ctx.device.type == "cuda":
            kw.setdefault("pin_memory", True)
        loader = _data.DataLoader(dataset, batch_size=batch_size, shuffle=False, **kw).get_data_loader(
            repeat=False, skip=skip, num_replicas=workers, rank=rank, shard_batches=True)
        # every rank runs the same number of iterations (ceil), so collectives never hang
        per_rank = math.ceil(len(dataset) / batch_size / workers)
        total = per_rank if max_batches is None or not (0 < max_batches <= per_rank) else max_batches
        it: Iterator[Any] = iter(loader)
        steps = skip
        last_ckpt = skip - 1
        op = core.DummySearcherOperation(1, rank == 0) if rank == 0 else None
        for batch_idx in range(skip, total):
            batch = next(it, None)
            if batch is not None:
                processor.process_batch(batch=batch, batch_idx=batch_idx)
            steps = batch_idx + 1
            if steps % checkpoint_interval == 0:
                processor.on_checkpoint_start()
                _checkpoint_progress(core_context, steps, output_uuid)
                last_ckpt = batch_idx
                if op is not None:
                    op.report_progress(min(1.0, steps * workers * batch_size / max(len(dataset), 1)))
                if core_context.preempt.should_preempt():
                    _reduce_metrics(ctx, core_context, steps)
                    return
        if steps - 1 > last_ckpt:
            processor.on_checkpoint_start()
            _checkpoint_progress(core_context, total, output_uuid)
        processor.on_finish()
        metrics = _reduce_metrics(ctx, core_context, steps)
        if info is not None and info.task_type == "TRIAL":
            # close the trial's searcher operation(s) so the master does not reschedule a task
            # whose work is done (every rank takes part: the ops are a collective)
            value = next(iter(metrics.values()), 0.0) if metrics else 0.0
            for op in core_context.searcher.operations():
                if rank == 0:
                    op.report_completed(float(value) if isinstance(value, (int, float)) else 0.0)
