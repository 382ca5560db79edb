"""``pytorch.Trainer`` and ``pytorch.init()`` (reference: ``harness/determined/pytorch/_trainer.py``).

``init()`` sets up the process group (RCCL on GPUs, gloo on CPU) when launched by
``torch.distributed.run``, then the Core API context, then a PyTorchTrialContext.
``Trainer.fit()`` runs the trial controller; on-cluster the training length comes from the
searcher, off-cluster from ``max_length``.
"""

import contextlib
import logging
import os
import random
from typing import Any, Dict, Iterator, Optional, Union

import numpy as np
import torch

from determined_amd import core
from determined_amd._info import get_cluster_info
from determined_amd.pytorch._context import PyTorchTrialContext
from determined_amd.pytorch._trial import Batch, Epoch, PyTorchTrial, TrainUnit, _PyTorchTrialController

logger = logging.getLogger("determined_amd.pytorch")


def _set_random_seeds(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.random.manual_seed(seed)


def _initialize_distributed_backend() -> Optional[core.DistributedContext]:
    size = int(os.environ.get("WORLD_SIZE", "1"))
    if size <= 1:
        return None
    import torch.distributed as dist

    if not dist.is_initialized():
        if torch.cuda.is_available():
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))  # RCCL over xGMI
        else:
            dist.init_process_group("gloo")
    return core.DistributedContext.from_torch_distributed()


def _period(d: Optional[Union[int, Dict[str, int]]], gbs: Optional[int]) -> TrainUnit:
    if d is None:
        return Batch(0)
    if isinstance(d, TrainUnit):
        return d
    return TrainUnit._from_config(d, gbs)


class Trainer:
    def __init__(self, trial: PyTorchTrial, context: PyTorchTrialContext) -> None:
        self._trial = trial
        self._context = context
        self._core = context._core
        self._info = get_cluster_info()
        self._local_training = self._info is None or self._info.task_type != "TRIAL"

    def configure_profiler(self, sync_timings: bool = True, enabled: bool = True, begin_on_batch: int = 0,
                           end_after_batch: Optional[int] = None) -> None:
        self._profiling_enabled = enabled

    def fit(self, checkpoint_period: Optional[TrainUnit] = None, validation_period: Optional[TrainUnit] = None,
            max_length: Optional[TrainUnit] = None, reporting_period: TrainUnit = Batch(100),
            average_training_metrics: Optional[bool] = None, test_mode: bool = False,
            searcher_metric_name: Optional[str] = None, checkpoint_policy: str = "best",
            latest_checkpoint: Optional[str] = None, step_zero_validation: bool = False,
            profiling_enabled: Optional[bool] = None) -> None:
        cfg = self._context._exp_conf or {}
        gbs = None
        try:
            gbs = self._context.get_global_batch_size()
        except (ValueError, KeyError):
            pass
        smaller_is_better = True
        steps_completed = 0
        if not self._local_training:
            assert self._info is not None
            if max_length is not None and not test_mode:
                logger.warning("max_length is ignored on-cluster: the searcher decides the training length")
            checkpoint_period = checkpoint_period or _period(cfg.get("min_checkpoint_period"), gbs)
            validation_period = validation_period or _period(cfg.get("min_validation_period"), gbs)
            reporting_period = Batch(int(cfg.get("scheduling_unit", 100)))
            searcher_metric_name = cfg.get("searcher", {}).get("metric", searcher_metric_name)
            smaller_is_better = bool(cfg.get("searcher", {}).get("smaller_is_better", True))
            checkpoint_policy = cfg.get("checkpoint_policy", checkpoint_policy)
            latest_checkpoint = self._info.latest_checkpoint
            steps_completed = self._info.trial._steps_completed
            step_zero_validation = bool(cfg.get("perform_initial_validation", step_zero_validation))
            if average_training_metrics is None:
                average_training_metrics = bool(cfg.get("optimizations", {}).get("average_training_metrics", True))
            if profiling_enabled is None:
                profiling_enabled = bool(cfg.get("profiling", {}).get("enabled", False))
        else:
            if max_length is None and not test_mode:
                raise ValueError("max_length is required for local training")
        controller_cls = getattr(self._trial, "trial_controller_class", None) or _PyTorchTrialController
        controller = controller_cls(
            trial_inst=self._trial,
            context=self._context,
            checkpoint_period=checkpoint_period or Batch(0),
            validation_period=validation_period or Batch(0),
            reporting_period=reporting_period,
            smaller_is_better=smaller_is_better,
            steps_completed=steps_completed,
            latest_checkpoint=latest_checkpoint,
            local_training=self._local_training,
            test_mode=test_mode,
            searcher_metric_name=searcher_metric_name,
            checkpoint_policy=checkpoint_policy,
            step_zero_validation=step_zero_validation,
            max_length=max_length,
            global_batch_size=gbs,
            profiling_enabled=bool(profiling_enabled),
            average_training_metrics=True if average_training_metrics is None else average_training_metrics,
        )
        controller.run()


@contextlib.contextmanager
def init(*, hparams: Optional[Dict[str, Any]] = None, exp_conf: Optional[Dict[str, Any]] = None,
         distributed: Optional[core.DistributedContext] = None, aggregation_frequency: int = 1,
         enable_tensorboard_logging: bool = True, checkpoint_storage: Any = None,
         ddp_bucket_mb: float = 16.0) -> Iterator[PyTorchTrialContext]:
    with _init_context(PyTorchTrialContext, hparams=hparams, exp_conf=exp_conf, distributed=distributed,
                       aggregation_frequency=aggregation_frequency,
                       enable_tensorboard_logging=enable_tensorboard_logging,
                       checkpoint_storage=checkpoint_storage, ddp_bucket_mb=ddp_bucket_mb) as ctx:
        yield ctx


@contextlib.contextmanager
def _init_context(context_cls: Any, *, hparams: Optional[Dict[str, Any]], exp_conf: Optional[Dict[str, Any]],
                  distributed: Optional[core.DistributedContext], aggregation_frequency: int,
                  enable_tensorboard_logging: bool, checkpoint_storage: Any, ddp_bucket_mb: float) -> Iterator[Any]:
    info = get_cluster_info()
    if distributed is None:
        distributed = _initialize_distributed_backend()
    if info is not None and info.task_type == "TRIAL":
        hparams = hparams if hparams is not None else info.trial.hparams
        exp_conf = exp_conf if exp_conf is not None else info.trial._config
        seed = info.trial.trial_seed
        steps_completed = info.trial._steps_completed
        opt = exp_conf.get("optimizations", {})
        aggregation_frequency = int(opt.get("aggregation_frequency", aggregation_frequency))
        avg_agg = bool(opt.get("average_aggregated_gradients", True))
        slots = int(exp_conf.get("resources", {}).get("slots_per_trial", 1))
        managed = True
    else:
        seed = int((exp_conf or {}).get("reproducibility", {}).get("experiment_seed") or 0)
        steps_completed = 0
        avg_agg = True
        slots = distributed.size if distributed is not None else 1
        managed = False
    _set_random_seeds(seed)
    num_gpus = 1 if torch.cuda.is_available() and slots > 0 else 0
    with core.init(distributed=distributed, checkpoint_storage=checkpoint_storage) as core_context:
        ctx = context_cls(core_context=core_context, trial_seed=seed, hparams=hparams,
                                  slots_per_trial=slots, num_gpus=num_gpus, exp_conf=exp_conf,
                                  aggregation_frequency=aggregation_frequency, steps_completed=steps_completed,
                                  managed_training=managed, debug_enabled=False,
                                  enable_tensorboard_logging=enable_tensorboard_logging,
                                  average_aggregated_gradients=avg_agg, ddp_bucket_mb=ddp_bucket_mb)
        yield ctx
