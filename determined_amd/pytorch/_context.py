"""PyTorchTrialContext (reference: ``harness/determined/pytorch/_pytorch_context.py``).

MI355X-native differences from the reference:
* ``wrap_model`` wraps GPU models in the native bucketed data-parallel engine
  (``parallel/ddp.py``: grads land in flat buckets, RCCL all-reduce overlaps backward),
  also for a single slot so fused optimizers always see stable gradient buffers;
* gradient aggregation (``optimizations.aggregation_frequency``) scales the loss instead of
  dividing every gradient afterwards, and skips collectives for non-final micro-batches;
* ``wrap_scaler`` accepts ``determined_amd.ops.DeviceGradScaler`` (no host sync per step) as
  well as ``torch.amp.GradScaler``.
"""

import contextlib
import logging
import pathlib
from typing import Any, Callable, Dict, Iterator, List, Optional, Union

import torch
from torch import nn

from determined_amd.pytorch import _data
from determined_amd.pytorch._lr_scheduler import LRScheduler
from determined_amd.pytorch._reducer import _PyTorchReducerContext

logger = logging.getLogger("determined_amd.pytorch")


class _SummaryWriter:
    """Minimal ``torch.utils.tensorboard.SummaryWriter`` (add_scalar[s]) on the native writer."""

    def __init__(self, logdir: str, rank: int) -> None:
        from determined_amd.tensorboard import EventFileWriter

        self._w = EventFileWriter(logdir, suffix=f".user.rank{rank}")

    def add_scalar(self, tag: str, value: Any, global_step: Optional[int] = None, *_: Any, **__: Any) -> None:
        if hasattr(value, "item"):
            value = value.item()
        self._w.add_scalar(tag, float(value), int(global_step or 0))

    def add_scalars(self, main_tag: str, values: Dict[str, Any], global_step: Optional[int] = None) -> None:
        for k, v in values.items():
            self.add_scalar(f"{main_tag}/{k}", v, global_step)

    def flush(self) -> None:
        self._w.flush()

    def close(self) -> None:
        self._w.close()


class PyTorchTrialContext(_PyTorchReducerContext):
    def __init__(self, core_context: Any, trial_seed: int, hparams: Optional[Dict[str, Any]],
                 slots_per_trial: int, num_gpus: int, exp_conf: Optional[Dict[str, Any]],
                 aggregation_frequency: int, steps_completed: int, managed_training: bool,
                 debug_enabled: bool, enable_tensorboard_logging: bool = True,
                 average_aggregated_gradients: bool = True, ddp_bucket_mb: float = 16.0) -> None:
        self._core = core_context
        self.distributed = core_context.distributed
        super().__init__(self.distributed.allgather)
        self._trial_seed = trial_seed
        self._hparams = hparams
        self._slots_per_trial = slots_per_trial
        self._num_gpus = num_gpus
        self._exp_conf = exp_conf
        self._aggregation_frequency = max(int(aggregation_frequency), 1)
        self._average_aggregated_gradients = average_aggregated_gradients
        self._steps_completed = steps_completed
        self._managed_training = managed_training
        self._debug = debug_enabled
        self._enable_tensorboard_logging = enable_tensorboard_logging
        self._ddp_bucket_mb = ddp_bucket_mb
        self.device = self._init_device()
        self.models: List[nn.Module] = []
        self.optimizers: List[torch.optim.Optimizer] = []
        self.lr_schedulers: List[LRScheduler] = []
        self._ddp: List[Any] = []
        self._ddp_finished_at = -1
        self._scaler: Any = None
        self._auto_amp = False
        self._current_batch_idx: Optional[int] = None
        self._epoch_len: Optional[int] = None
        self._stop_requested = False
        self._tbd_writer: Optional[_SummaryWriter] = None
        self.profiler: Any = None
        self._main_model: Optional[nn.Module] = None
        self._is_pre_trainer = False
        from determined_amd.pytorch._experimental import PyTorchExperimentalContext

        self.experimental = PyTorchExperimentalContext(self)

    # -- basic info --------------------------------------------------------------------------
    def _init_device(self) -> torch.device:
        if self._num_gpus > 0 and torch.cuda.is_available():
            d = torch.device("cuda", self.distributed.local_rank % max(torch.cuda.device_count(), 1))
            torch.cuda.set_device(d)
            return d
        return torch.device("cpu")

    def get_hparams(self) -> Dict[str, Any]:
        if self._hparams is None:
            raise ValueError("hparams are not available in this context")
        return self._hparams

    def get_hparam(self, name: str) -> Any:
        hp = self.get_hparams()
        if name not in hp:
            raise ValueError(f"could not find hyperparameter {name!r} (available: {sorted(hp)})")
        return hp[name]

    def get_experiment_config(self) -> Dict[str, Any]:
        if self._exp_conf is None:
            raise ValueError("experiment config is not available in this context")
        return self._exp_conf

    def get_global_batch_size(self) -> int:
        return int(self.get_hparam("global_batch_size"))

    def get_per_slot_batch_size(self) -> int:
        gbs = self.get_global_batch_size()
        n = max(self.distributed.size, 1)
        if gbs % n:
            logger.warning(f"global_batch_size {gbs} is not divisible by {n} slots; rounding down")
        return max(gbs // n, 1)

    def get_data_config(self) -> Dict[str, Any]:
        return (self._exp_conf or {}).get("data", {})

    def get_experiment_id(self) -> int:
        info = self._core.info
        return info.trial.experiment_id if info is not None else 0

    def get_trial_id(self) -> int:
        info = self._core.info
        return info.trial.trial_id if info is not None else 0

    def get_trial_seed(self) -> int:
        return self._trial_seed

    def get_initial_batch(self) -> int:
        return self._steps_completed

    def get_stop_requested(self) -> bool:
        return self._stop_requested

    def set_stop_requested(self, stop_requested: bool) -> None:
        self._stop_requested = bool(stop_requested)

    def set_enable_tensorboard_logging(self, enable: bool) -> None:
        self._enable_tensorboard_logging = enable

    def get_enable_tensorboard_logging(self) -> bool:
        return self._enable_tensorboard_logging

    def current_train_epoch(self) -> int:
        if self._epoch_len is None or self._current_batch_idx is None:
            raise RuntimeError("training has not started")
        return self._current_batch_idx // self._epoch_len

    def current_train_batch(self) -> int:
        if self._current_batch_idx is None:
            raise RuntimeError("training has not started")
        return self._current_batch_idx

    def is_epoch_start(self) -> bool:
        return self._epoch_len is not None and self._current_batch_idx is not None and \
            self._current_batch_idx % self._epoch_len == 0

    def is_epoch_end(self) -> bool:
        return self._epoch_len is not None and self._current_batch_idx is not None and \
            self._current_batch_idx % self._epoch_len == self._epoch_len - 1

    def get_tensorboard_path(self) -> pathlib.Path:
        return self._core.train.get_tensorboard_path()

    def get_tensorboard_writer(self) -> _SummaryWriter:
        if self._tbd_writer is None:
            try:
                path = str(self.get_tensorboard_path())
            except Exception:
                path = "/tmp/tensorboard/local"
            self._tbd_writer = _SummaryWriter(path, self.distributed.rank)
        return self._tbd_writer

    # -- wrapping ----------------------------------------------------------------------------
    def wrap_model(self, model: nn.Module) -> nn.Module:
        model = model.to(self.device)
        if self.device.type == "cuda" or self.distributed.size > 1:
            from determined_amd.parallel.ddp import DistributedDataParallel

            wrapped = DistributedDataParallel(model, bucket_cap_mb=self._ddp_bucket_mb)
            self._ddp.append(wrapped)
            if self.experimental._auto_amp:
                wrapped = self.autocast_forward_pass(wrapped, dtype=self._amp_dtype())
            self.models.append(wrapped)
            if self._main_model is None:
                self._main_model = wrapped
            return wrapped
        if self.experimental._auto_amp:
            model = self.autocast_forward_pass(model, dtype=self._amp_dtype())
        self.models.append(model)
        if self._main_model is None:
            self._main_model = model
        return model

    def wrap_optimizer(self, optimizer: torch.optim.Optimizer, backward_passes_per_step: int = 1,
                       fp16_compression: bool = False, average_aggregated_gradients: Optional[bool] = None
                       ) -> torch.optim.Optimizer:
        if average_aggregated_gradients is not None:
            self._average_aggregated_gradients = average_aggregated_gradients
        self.optimizers.append(optimizer)
        return optimizer

    def wrap_lr_scheduler(self, lr_scheduler: Any, step_mode: LRScheduler.StepMode, frequency: int = 1) -> Any:
        wrapped = LRScheduler(lr_scheduler, step_mode, frequency)
        self.lr_schedulers.append(wrapped)
        return lr_scheduler

    def wrap_scaler(self, scaler: Any) -> Any:
        self._scaler = scaler
        return scaler

    def wrap_reducer(self, reducer: Any, name: Optional[str] = None, for_training: bool = True,
                     for_validation: bool = True) -> Any:
        return super().wrap_reducer(reducer, name, for_training, for_validation)

    def autocast_forward_pass(self, to_wrap: nn.Module, dtype: torch.dtype = torch.bfloat16) -> nn.Module:
        dev = self.device.type
        orig = to_wrap.forward

        def forward(*a: Any, **kw: Any) -> Any:
            with torch.autocast(dev, dtype=dtype):
                return orig(*a, **kw)

        to_wrap.forward = forward  # type: ignore
        return to_wrap

    def _amp_dtype(self) -> torch.dtype:
        """``experimental.use_amp()``: fp16 (with loss scaling) on the GPU, bf16 on the CPU."""
        return torch.float16 if self.device.type == "cuda" else torch.bfloat16

    def configure_apex_amp(self, *args: Any, **kwargs: Any) -> Any:
        raise RuntimeError("NVIDIA apex is not available on ROCm; use wrap_scaler(DeviceGradScaler()) or bf16")

    def set_profiler(self, *args: Any, **kwargs: Any) -> None:
        """Attach a ``torch.profiler.profile`` (entered around every train_batch)."""
        self.profiler = torch.profiler.profile(*args, **kwargs)

    def to_device(self, data: Any) -> Any:
        return _data.to_device(data, self.device)

    # -- backward / step ---------------------------------------------------------------------
    def _should_communicate_and_update(self) -> bool:
        if self._current_batch_idx is None:
            return True
        return (self._current_batch_idx + 1) % self._aggregation_frequency == 0

    @contextlib.contextmanager
    def _no_sync(self) -> Iterator[None]:
        with contextlib.ExitStack() as st:
            for d in self._ddp:
                st.enter_context(d.no_sync())
            yield

    def backward(self, loss: torch.Tensor, gradient: Optional[torch.Tensor] = None, retain_graph: bool = False,
                 create_graph: bool = False) -> None:
        if self._aggregation_frequency > 1 and self._average_aggregated_gradients:
            loss = loss / self._aggregation_frequency
        if self._scaler is not None and self.experimental._auto_amp:  # manual scalers: the trial scales
            loss = self._scaler.scale(loss)
        if self._should_communicate_and_update():
            loss.backward(gradient=gradient, retain_graph=retain_graph, create_graph=create_graph)
        else:
            with self._no_sync():
                loss.backward(gradient=gradient, retain_graph=retain_graph, create_graph=create_graph)

    def _finish_grads(self) -> None:
        idx = self._current_batch_idx if self._current_batch_idx is not None else -2
        if self._ddp_finished_at == idx and idx >= 0:
            return
        for d in self._ddp:
            d.finish()
        self._ddp_finished_at = idx

    def step_optimizer(self, optimizer: torch.optim.Optimizer,
                       clip_grads: Optional[Callable[[Iterator], None]] = None, auto_zero_grads: bool = True,
                       scaler: Optional[Any] = None) -> None:
        if not self._should_communicate_and_update():
            return
        self._finish_grads()
        # the wrapped scaler steps automatically only under experimental.use_amp(); a manual scaler
        # is passed in (``step_optimizer(opt, scaler=s)``) and unscaled by the trial before clipping
        if scaler is None and self.experimental._auto_amp:
            scaler = self._scaler
        if clip_grads is not None:
            if self._scaler is not None and self.experimental._auto_amp:
                self._scaler.unscale_(optimizer)
            params = [p for g in optimizer.param_groups for p in g["params"]]
            clip_grads(params)
        if scaler is not None:
            scaler.step(optimizer)
        else:
            optimizer.step()
        if auto_zero_grads:
            self._zero_grads(optimizer)

    def _zero_grads(self, optimizer: torch.optim.Optimizer) -> None:
        owned = set()
        for d in self._ddp:
            d.zero_grad()
            owned.update(id(p) for p in d.module.parameters())
        rest = [p for g in optimizer.param_groups for p in g["params"] if id(p) not in owned]
        for p in rest:
            p.grad = None

    @property
    def _main(self) -> Optional[nn.Module]:
        return self._main_model
