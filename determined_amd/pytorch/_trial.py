"""PyTorchTrial and its controller (reference: ``harness/determined/pytorch/_pytorch_trial.py``).

The controller walks the searcher's operations (train to an absolute length, validate, report
the searcher metric), interleaving validation / checkpoint / metric-report boundaries and
preemption checks exactly like the reference.  MI355X-native differences:
* per-batch training metrics stay on the GPU; they are stacked, averaged and all-reduced ONCE
  per reporting period (the reference converts every batch's metrics with ``.cpu()``, a host
  sync per step: ``_pytorch_trial.py:_train_batch``);
* checkpoints are written without pickled controller state (``trial_state.json``) and RNG
  states are stored as tensors/lists, so they load with ``torch.load(weights_only=True)``.
"""

import abc
import contextlib
import enum
import json
import logging
import math
import os
import pathlib
import random
import shutil
import sys
import time
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple, Type, Union

import numpy as np
import torch

from determined_amd import core
from determined_amd.pytorch import _data
from determined_amd.pytorch._callback import PyTorchCallback
from determined_amd.pytorch._context import PyTorchTrialContext
from determined_amd.pytorch._lr_scheduler import LRScheduler
from determined_amd.pytorch._reducer import Reducer, _simple_reduce_metrics

logger = logging.getLogger("determined_amd.pytorch")

CHECKPOINT_FORMAT = "determined_amd-pytorch-v1"


class TrainUnit:
    def __init__(self, value: int) -> None:
        self.value = int(value)

    @staticmethod
    def _from_searcher_unit(length: int, unit: Optional[core.Unit], global_batch_size: Optional[int] = None
                            ) -> "TrainUnit":
        if unit == core.Unit.EPOCHS:
            return Epoch(length)
        if unit == core.Unit.RECORDS:
            if not global_batch_size:
                raise ValueError("record lengths need global_batch_size")
            return Batch(math.ceil(length / global_batch_size))
        return Batch(length)

    @staticmethod
    def _from_values(batches: Optional[int] = None, records: Optional[int] = None, epochs: Optional[int] = None,
                     global_batch_size: Optional[int] = None) -> "TrainUnit":
        if sum(x is not None for x in (batches, records, epochs)) != 1:
            raise ValueError("exactly one of batches/records/epochs must be set")
        if batches is not None:
            return Batch(batches)
        if records is not None:
            if not global_batch_size:
                raise ValueError("record lengths need global_batch_size")
            return Batch(math.ceil(records / global_batch_size))
        return Epoch(int(epochs))  # type: ignore

    @staticmethod
    def _from_config(d: Union[int, Dict[str, int]], global_batch_size: Optional[int]) -> "TrainUnit":
        if isinstance(d, int):
            return Batch(d)
        return TrainUnit._from_values(**{k: v for k, v in d.items()}, global_batch_size=global_batch_size)

    def should_stop(self, step_num: int) -> bool:
        return self.value > 0 and step_num >= self.value and step_num % self.value == 0

    def __repr__(self) -> str:
        return f"{type(self).__name__}({self.value})"


class Epoch(TrainUnit):
    pass


class Batch(TrainUnit):
    pass


class _TrainBoundaryType(enum.Enum):
    CHECKPOINT = "CHECKPOINT"
    REPORT = "REPORT"
    VALIDATE = "VALIDATE"
    TRAIN = "TRAIN"


class _TrainBoundary:
    def __init__(self, step_type: _TrainBoundaryType, unit: TrainUnit) -> None:
        self.step_type = step_type
        self.unit = unit
        self.limit_reached = False


class ShouldExit(Exception):
    def __init__(self, skip_exit_checkpoint: bool = False) -> None:
        super().__init__()
        self.skip_exit_checkpoint = skip_exit_checkpoint


class _TrialState:
    def __init__(self, trial_id: int = 0, last_ckpt: int = 0, step_id: int = 0, last_val: int = 0,
                 batches_trained: int = 0, epochs_trained: int = 0) -> None:
        self.trial_id = trial_id
        self.last_ckpt = last_ckpt
        self.step_id = step_id
        self.last_val = last_val
        self.batches_trained = batches_trained
        self.epochs_trained = epochs_trained

    def to_dict(self) -> Dict[str, int]:
        return dict(vars(self))


class PyTorchTrial(metaclass=abc.ABCMeta):
    """Subclass and implement ``train_batch``, ``build_training_data_loader``,
    ``build_validation_data_loader`` and ``evaluate_batch`` (or ``evaluate_full_dataset``)."""

    trial_context_class = PyTorchTrialContext

    def __init__(self, context: PyTorchTrialContext) -> None:
        pass

    @abc.abstractmethod
    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Union[torch.Tensor, Dict[str, Any]]:
        pass

    @abc.abstractmethod
    def build_training_data_loader(self) -> Any:
        pass

    @abc.abstractmethod
    def build_validation_data_loader(self) -> Any:
        pass

    def build_callbacks(self) -> Dict[str, PyTorchCallback]:
        return {}

    def evaluate_batch(self, batch: Any, batch_idx: int) -> Dict[str, Any]:
        raise NotImplementedError

    def evaluation_reducer(self) -> Union[Reducer, Dict[str, Reducer]]:
        return Reducer.AVG

    def evaluate_full_dataset(self, data_loader: Any) -> Dict[str, Any]:
        raise NotImplementedError

    def get_batch_length(self, batch: Any) -> int:
        return _data.data_length(batch)


def _rng_state() -> Dict[str, Any]:
    np_state = np.random.get_state()
    st: Dict[str, Any] = {
        "cpu_rng_state": torch.random.get_rng_state(),
        "np_rng_state": {"key": np_state[0], "pos": int(np_state[2]), "has_gauss": int(np_state[3]),
                         "cached_gaussian": float(np_state[4]), "state": torch.from_numpy(np_state[1].astype(np.int64))},
        "random_rng_state": [random.getstate()[0], list(random.getstate()[1]), random.getstate()[2]],
    }
    if torch.cuda.is_available():
        st["gpu_rng_state"] = torch.cuda.get_rng_state()
    return st


def _set_rng_state(st: Dict[str, Any]) -> None:
    torch.random.set_rng_state(st["cpu_rng_state"])
    n = st["np_rng_state"]
    np.random.set_state((n["key"], n["state"].numpy().astype(np.uint32), n["pos"], n["has_gauss"],
                         n["cached_gaussian"]))
    r = st["random_rng_state"]
    random.setstate((r[0], tuple(r[1]), r[2]))
    if torch.cuda.is_available() and "gpu_rng_state" in st:
        torch.cuda.set_rng_state(st["gpu_rng_state"])


def _set_random_seeds(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.random.manual_seed(seed)


class _PyTorchTrialController:
    def __init__(self, trial_inst: PyTorchTrial, context: PyTorchTrialContext, checkpoint_period: TrainUnit,
                 validation_period: TrainUnit, reporting_period: TrainUnit, smaller_is_better: bool,
                 steps_completed: int, latest_checkpoint: Optional[str], local_training: bool, test_mode: bool,
                 searcher_metric_name: Optional[str], checkpoint_policy: str, step_zero_validation: bool,
                 max_length: Optional[TrainUnit], global_batch_size: Optional[int], profiling_enabled: bool = False,
                 average_training_metrics: bool = True) -> None:
        self.trial = trial_inst
        self.context = context
        self.core_context = context._core
        self.is_chief = context.distributed.rank == 0
        self.checkpoint_period = checkpoint_period
        self.validation_period = validation_period
        self.reporting_period = reporting_period
        self.smaller_is_better = smaller_is_better
        self.steps_completed = steps_completed
        self.latest_checkpoint = latest_checkpoint
        self.local_training = local_training
        self.test_mode = test_mode
        self.searcher_metric_name = searcher_metric_name
        self.checkpoint_policy = checkpoint_policy
        self.step_zero_validation = step_zero_validation
        self.max_length = max_length
        self.global_batch_size = global_batch_size
        self.profiling_enabled = profiling_enabled
        self.average_training_metrics = average_training_metrics
        self.searcher_unit = self.core_context.searcher.get_configured_units()
        self.callbacks = self.trial.build_callbacks()
        self.state = _TrialState(trial_id=context.get_trial_id())
        self._best_val: Optional[float] = None
        self._val_from_previous_run = self.core_context.train._get_last_validation()

    # -- data --------------------------------------------------------------------------------
    def _set_data_loaders(self) -> None:
        dist = self.context.distributed
        tl = self.trial.build_training_data_loader()
        skip = self.state.batches_trained
        if isinstance(tl, _data.DataLoader):
            self._train_loader_len = len(tl) // dist.size if dist.size > 1 else len(tl)
            self.training_loader = tl.get_data_loader(repeat=True, skip=skip, num_replicas=dist.size,
                                                      rank=dist.rank, seed=self.context.get_trial_seed())
        else:
            if not self.context.experimental._data_repro_checks_disabled:
                raise RuntimeError(_data.dataset_repro_message("build_training_data_loader", tl))
            self._train_loader_len = len(tl)
            self.training_loader = _repeat(tl, skip)
        self.context._epoch_len = max(self._train_loader_len, 1)
        vl = self.trial.build_validation_data_loader()
        if isinstance(vl, _data.DataLoader):
            # every rank validates a disjoint round-robin share of the batches (no padding)
            self.validation_loader = vl.get_data_loader(repeat=False, num_replicas=dist.size, rank=dist.rank,
                                                        shard_batches=True)
            self._val_shard = (1, 0)
        else:
            if not self.context.experimental._data_repro_checks_disabled:
                raise RuntimeError(_data.dataset_repro_message("build_validation_data_loader", vl))
            self.validation_loader = vl
            self._val_shard = (1, 0)

    def _make_training_enumerator(self) -> Iterator:
        """Yields ``(batch_idx, batch)`` pairs for ``_train_with_boundaries``."""
        return enumerate(iter(self.training_loader), start=self.state.batches_trained)

    def _iter_eval_metrics(self) -> Iterator[Dict[str, Any]]:
        """Runs ``evaluate_batch`` over this rank's share of the validation data."""
        n_shards, shard = self._val_shard
        for idx, batch in enumerate(self.validation_loader):
            if idx % n_shards != shard:
                continue
            if self.context.experimental._auto_to_device:
                batch = self.context.to_device(batch)
            yield self.trial.evaluate_batch(batch=batch, batch_idx=idx)

    # -- checkpointing -----------------------------------------------------------------------
    def _save(self, path: pathlib.Path) -> None:
        path.mkdir(parents=True, exist_ok=True)
        ckpt: Dict[str, Any] = {
            "models_state_dict": [m.state_dict() for m in self.context.models],
            "optimizers_state_dict": [o.state_dict() for o in self.context.optimizers],
            "lr_schedulers_state_dict": [s.state_dict() for s in self.context.lr_schedulers],
            "callbacks": {n: cb.state_dict() for n, cb in self.callbacks.items()},
            "rng_state": _rng_state(),
        }
        if self.context._scaler is not None and hasattr(self.context._scaler, "state_dict"):
            ckpt["scaler_state_dict"] = self.context._scaler.state_dict()
        for cb in self.callbacks.values():
            cb.on_checkpoint_save_start(ckpt)
        torch.save(ckpt, path / "state_dict.pth")
        with open(path / "trial_state.json", "w") as f:
            json.dump(self.state.to_dict(), f)
        cls = type(self.trial)
        try:
            exp_conf: Optional[Dict[str, Any]] = self.context.get_experiment_config()
            hparams: Optional[Dict[str, Any]] = self.context.get_hparams()
        except ValueError:
            exp_conf, hparams = None, None
        with open(path / "load_data.json", "w") as f:
            json.dump({"trial_type": "PyTorchTrial", "experiment_config": exp_conf, "hparams": hparams,
                       "trial_cls_spec": f"{cls.__module__}:{cls.__qualname__}", "is_trainer": True,
                       "format": CHECKPOINT_FORMAT}, f, default=str)
        code_dir = os.environ.get("DET_MODEL_DEF_DIR")
        if code_dir and os.path.isdir(code_dir):
            shutil.copytree(code_dir, path / "code", dirs_exist_ok=True,
                            ignore=shutil.ignore_patterns("__pycache__", "*.pyc"))
        for cb in self.callbacks.values():
            cb.on_checkpoint_end(str(path))
            cb.on_checkpoint_write_end(str(path))

    def _load(self, load_path: pathlib.Path) -> None:
        sd_path = load_path / "state_dict.pth"
        if not sd_path.exists():
            raise FileNotFoundError(f"no state_dict.pth in checkpoint {load_path}")
        ckpt = torch.load(str(sd_path), map_location="cpu", weights_only=True)
        for cb in self.callbacks.values():
            cb.on_checkpoint_load_start(ckpt)
        for model, sd in zip(self.context.models, ckpt["models_state_dict"]):
            target = model.module if hasattr(model, "module") else model
            sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
            target.load_state_dict(sd)
        for opt, sd in zip(self.context.optimizers, ckpt["optimizers_state_dict"]):
            opt.load_state_dict(sd)
        for sch, sd in zip(self.context.lr_schedulers, ckpt.get("lr_schedulers_state_dict", [])):
            sch.load_state_dict(sd)
        if "scaler_state_dict" in ckpt and self.context._scaler is not None:
            self.context._scaler.load_state_dict(ckpt["scaler_state_dict"])
        for name, cb in self.callbacks.items():
            if name in ckpt.get("callbacks", {}):
                cb.load_state_dict(ckpt["callbacks"][name])
        if "rng_state" in ckpt:
            _set_rng_state(ckpt["rng_state"])
        ts = load_path / "trial_state.json"
        if ts.exists():
            st = json.loads(ts.read_text())
            self.state = _TrialState(**{k: v for k, v in st.items() if k in vars(_TrialState())})
            if self.state.trial_id != self.context.get_trial_id():
                # warm start from another trial's checkpoint: keep weights, restart counters
                self.state = _TrialState(trial_id=self.context.get_trial_id())
        else:
            self.state = _TrialState(trial_id=self.context.get_trial_id(), batches_trained=self.steps_completed)

    def _checkpoint(self, already_exiting: bool) -> None:
        if self.is_chief:
            self.core_context.train.set_status("checkpointing")
        self.state.last_ckpt = self.state.batches_trained
        metadata = {"steps_completed": self.state.batches_trained, "framework": f"torch-{torch.__version__}",
                    "format": CHECKPOINT_FORMAT}
        uuid = None
        if self.is_chief:
            with self.core_context.checkpoint.store_path(metadata) as (path, storage_id):
                self._save(path)
            uuid = storage_id
            for cb in self.callbacks.values():
                cb.on_checkpoint_upload_end(uuid)
        self.context.distributed.broadcast(uuid)  # everyone waits for the chief's checkpoint

    # -- training ----------------------------------------------------------------------------
    def _stop_requested(self) -> None:
        if self.context.get_stop_requested():
            raise ShouldExit()
        if self.core_context.preempt.should_preempt():
            raise ShouldExit()

    def _report_progress(self, op: Any) -> None:
        if not self.is_chief or op._completed:
            return
        if self.searcher_unit == core.Unit.EPOCHS:
            op.report_progress(self.state.batches_trained / max(self.context._epoch_len or 1, 1))
        elif self.searcher_unit == core.Unit.RECORDS and self.global_batch_size:
            op.report_progress(self.state.batches_trained * self.global_batch_size)
        else:
            op.report_progress(self.state.batches_trained)

    def _steps_until_complete(self, unit: TrainUnit) -> int:
        if isinstance(unit, Epoch):
            return unit.value * (self.context._epoch_len or 1) - self.state.batches_trained
        return unit.value - self.state.batches_trained

    def _auto_step_lr_schedulers(self, batch_idx: int) -> None:
        if not self.context._should_communicate_and_update():
            return
        agg = self.context._aggregation_frequency
        for s in self.context.lr_schedulers:
            if s._step_mode == LRScheduler.StepMode.STEP_EVERY_BATCH:
                for i in range(batch_idx - agg + 1, batch_idx + 1):
                    if (i + 1) % s._frequency == 0:
                        s.step()
            elif s._step_mode == LRScheduler.StepMode.STEP_EVERY_OPTIMIZER_STEP:
                if (batch_idx + 1) % s._frequency == 0:
                    s.step()
            elif s._step_mode == LRScheduler.StepMode.STEP_EVERY_EPOCH:
                el = self.context._epoch_len or 1
                e0, e1 = batch_idx // el, (batch_idx + agg) // el
                for e in range(e0, e1):
                    if (e + 1) % s._frequency == 0:
                        s.step()

    def _train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, Any]:
        if self.context.experimental._auto_to_device:
            batch = self.context.to_device(batch)
        with contextlib.ExitStack() as st:
            if self.context.profiler is not None:
                st.enter_context(self.context.profiler)
            out = self.trial.train_batch(batch=batch, epoch_idx=epoch_idx, batch_idx=batch_idx)
            if self.context.profiler is not None:
                self.context.profiler.step()
        if self.context._scaler is not None and self.context.experimental._auto_amp and \
                self.context._should_communicate_and_update():
            self.context._scaler.update()
        if isinstance(out, torch.Tensor):
            out = {"loss": out}
        if not isinstance(out, dict):
            raise TypeError("train_batch must return a dict of metrics or a loss tensor")
        self._auto_step_lr_schedulers(batch_idx)
        return {k: (v.detach() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}

    def _aggregate_training_metrics(self, per_batch: List[Dict[str, Any]]) -> Dict[str, Any]:
        """One stack + mean per metric on device, one cross-rank all-reduce, one D2H copy."""
        if not per_batch:
            return {"avg_metrics": {}, "batch_metrics": []}
        keys = list(per_batch[0].keys())
        dev = self.context.device
        tensor_keys = [k for k in keys if all(isinstance(b.get(k), (torch.Tensor, int, float)) for b in per_batch)]
        stacked = None
        if tensor_keys:
            stacked = torch.stack([torch.stack([torch.as_tensor(b[k], device=dev, dtype=torch.float32).reshape(())
                                                for k in tensor_keys]) for b in per_batch])  # [B, K]
            avg = stacked.mean(0)
            dist = self.context.distributed
            if dist.size > 1 and self.average_training_metrics:
                import torch.distributed as tdist

                if tdist.is_initialized():
                    avg = avg.clone()
                    tdist.all_reduce(avg)
                    avg /= dist.size
            avg_host = avg.cpu().tolist()
            batch_host = stacked.cpu().tolist()
        else:
            avg_host, batch_host = [], [[] for _ in per_batch]
        avg_metrics = dict(zip(tensor_keys, avg_host))
        batch_metrics = [dict(zip(tensor_keys, row)) for row in batch_host]
        return {"avg_metrics": avg_metrics, "batch_metrics": batch_metrics}

    def _train_with_boundaries(self, enumerator: Iterator, boundaries: List[_TrainBoundary]) -> List[Dict[str, Any]]:
        if self.is_chief:
            self.core_context.train.set_status("training")
        for m in self.context.models:
            m.train()
        self.context.reset_reducers()
        metrics: List[Dict[str, Any]] = []
        epoch_len = self.context._epoch_len or 1
        for batch_idx, batch in enumerator:
            epoch_idx, in_epoch = divmod(batch_idx, epoch_len)
            self.context._current_batch_idx = batch_idx
            if in_epoch == 0:
                for cb in self.callbacks.values():
                    cb.on_training_epoch_start(epoch_idx)
            metrics.append(self._train_batch(batch, epoch_idx, batch_idx))
            self.state.batches_trained += 1
            if in_epoch == epoch_len - 1:
                self.state.epochs_trained += 1
                for cb in self.callbacks.values():
                    cb.on_training_epoch_end(epoch_idx)
            for b in boundaries:
                if isinstance(b.unit, Batch) and b.unit.should_stop(batch_idx + 1):
                    b.limit_reached = True
                if isinstance(b.unit, Epoch) and in_epoch == epoch_len - 1 and b.unit.should_stop(epoch_idx + 1):
                    b.limit_reached = True
                if b.step_type == _TrainBoundaryType.TRAIN and self.test_mode:
                    b.limit_reached = True
            if any(b.limit_reached for b in boundaries):
                return metrics
        return metrics

    def _train_for_op(self, op: Any, boundaries: List[_TrainBoundary]) -> None:
        if self.test_mode:
            length: TrainUnit = Batch(1)
        elif self.local_training:
            length = self.max_length  # type: ignore
        else:
            length = TrainUnit._from_searcher_unit(op.length, self.searcher_unit, self.global_batch_size)
        while self._steps_until_complete(length) > 0:
            per_batch = self._train_with_boundaries(self.training_enumerator, boundaries)
            m = self._aggregate_training_metrics(per_batch)
            if self.context.device.type == "cuda":
                from determined_amd import ops

                ops.conv_health_check(self.context.device)  # stream-K conv hand-off time-outs raise here
            if self.is_chief and m["avg_metrics"]:
                self.core_context.train.report_training_metrics(self.state.batches_trained, m["avg_metrics"],
                                                                m["batch_metrics"])
            for cb in self.callbacks.values():
                cb.on_training_workload_end(avg_metrics=m["avg_metrics"], batch_metrics=m["batch_metrics"])
            reported = False
            for b in boundaries:
                if not b.limit_reached:
                    continue
                if b.step_type in (_TrainBoundaryType.TRAIN, _TrainBoundaryType.REPORT):
                    if not reported:
                        self._report_progress(op)
                        reported = True
                elif b.step_type == _TrainBoundaryType.VALIDATE:
                    if not self._validation_is_current():
                        self._validate(op)
                elif b.step_type == _TrainBoundaryType.CHECKPOINT:
                    if not self._checkpoint_is_current():
                        self._checkpoint(already_exiting=False)
                b.limit_reached = False
                self._stop_requested()
            if self.test_mode:
                break
        if not self._validation_is_current():
            self._validate(op)
        if not self._checkpoint_is_current():
            self._checkpoint(already_exiting=False)
        if self.is_chief and not self.test_mode and not op._completed:
            raise ShouldExit(skip_exit_checkpoint=True)

    def _checkpoint_is_current(self) -> bool:
        return self.state.last_ckpt == self.state.batches_trained

    def _validation_is_current(self) -> bool:
        return self.state.last_val == self.state.batches_trained

    # -- validation --------------------------------------------------------------------------
    def _evaluate_batch_defined(self) -> bool:
        return type(self.trial).evaluate_batch is not PyTorchTrial.evaluate_batch

    @torch.no_grad()
    def _validate(self, op: Any = None) -> Dict[str, Any]:
        if self.is_chief:
            self.core_context.train.set_status("validating")
        for m in self.context.models:
            m.eval()
        for cb in self.callbacks.values():
            cb.on_validation_start()
            cb.on_validation_epoch_start()
        self.context.reset_reducers()
        dist = self.context.distributed
        if self._evaluate_batch_defined():
            sums: Dict[str, List[Any]] = {}
            num = 0
            outputs = []
            for vm in self._iter_eval_metrics():
                if not isinstance(vm, dict):
                    raise TypeError("evaluate_batch must return a dict of metric names to values")
                outputs.append(vm)
                for k, v in vm.items():
                    sums.setdefault(k, []).append(v.detach() if isinstance(v, torch.Tensor) else v)
                num += 1
            per_slot = {}
            for k, vals in sums.items():
                if vals and all(isinstance(v, torch.Tensor) and v.numel() == 1 for v in vals):
                    per_slot[k] = torch.stack([v.float().reshape(()) for v in vals]).mean().item()
                else:
                    per_slot[k] = _simple_reduce_metrics(Reducer.AVG, [
                        v.cpu().numpy() if isinstance(v, torch.Tensor) else v for v in vals])
            gathered = dist.allgather((per_slot, num))
            reducer = self.trial.evaluation_reducer()
            metrics: Dict[str, Any] = {}
            keys = gathered[0][0].keys()
            for k in keys:
                red = reducer[k] if isinstance(reducer, dict) else reducer
                vals = [g[0][k] for g in gathered if g[1] > 0]
                counts = [g[1] for g in gathered if g[1] > 0]
                val = _simple_reduce_metrics(red, vals, counts if red == Reducer.AVG else None)
                metrics[k] = val.item() if hasattr(val, "item") and np.ndim(val) == 0 else val
            metrics.update(self.context.reduce_metrics(for_training=False))
            for cb in self.callbacks.values():
                cb.on_validation_epoch_end(outputs)
        else:
            metrics = {}
            if self.is_chief:
                metrics = self.trial.evaluate_full_dataset(data_loader=self.validation_loader)
                metrics = {k: (v.item() if isinstance(v, torch.Tensor) and v.numel() == 1 else v)
                           for k, v in metrics.items()}
            metrics = dist.broadcast(metrics)
        self.state.last_val = self.state.batches_trained
        if self.is_chief:
            self.core_context.train.report_validation_metrics(self.state.batches_trained, metrics)
        for cb in self.callbacks.values():
            cb.on_validation_end(metrics)
        for m in self.context.models:
            m.train()
        searcher_metric = None
        if self.searcher_metric_name is not None:
            if self.searcher_metric_name not in metrics:
                raise RuntimeError(f"searcher metric {self.searcher_metric_name!r} not in validation metrics "
                                   f"{sorted(metrics)}")
            searcher_metric = metrics[self.searcher_metric_name]
            if not isinstance(searcher_metric, (int, float, np.floating, np.integer)):
                raise RuntimeError(f"searcher metric {self.searcher_metric_name!r} must be a scalar")
        # checkpoint policy
        if self.checkpoint_policy == "all" or (self.checkpoint_policy == "best" and searcher_metric is not None
                                               and self._is_best(float(searcher_metric))):
            if not self._checkpoint_is_current():
                self._checkpoint(already_exiting=False)
        if op is not None and self.is_chief and not op._completed and not self.test_mode:
            length = self.max_length if self.local_training else TrainUnit._from_searcher_unit(
                op.length, self.searcher_unit, self.global_batch_size)
            if length is not None and self._steps_until_complete(length) <= 0:
                op.report_completed(float(searcher_metric) if searcher_metric is not None else 0.0)
        return metrics

    def _is_best(self, v: float) -> bool:
        prev = self._best_val
        if not self.local_training:
            best = self.core_context.train.get_experiment_best_validation() if self.is_chief else None
            prev = best if best is not None else prev
        better = prev is None or (v < prev if self.smaller_is_better else v > prev)
        if better:
            self._best_val = v
        return bool(self.context.distributed.broadcast(better))

    # -- run ---------------------------------------------------------------------------------
    def run(self) -> None:
        with contextlib.ExitStack() as es:
            for cb in self.callbacks.values():
                cb.on_trial_startup(self.steps_completed, self.latest_checkpoint)
                es.callback(cb.on_trial_shutdown)
            if self.latest_checkpoint is not None:
                logger.info(f"restoring trial from checkpoint {self.latest_checkpoint}")
                with self.core_context.checkpoint.restore_path(self.latest_checkpoint) as p:
                    self._load(pathlib.Path(p))
            self._set_data_loaders()
            self.training_enumerator = self._make_training_enumerator()
            for cb in self.callbacks.values():
                cb.on_training_start()
            if self.profiling_enabled:
                self.core_context.profiler.on()
            self._run()

    def _run(self) -> None:
        try:
            if self.step_zero_validation and self._val_from_previous_run is None and self.state.batches_trained == 0:
                self._validate()
            if self.local_training:
                ops = iter([core.DummySearcherOperation(self.max_length.value if self.max_length else 1,
                                                        self.is_chief)])
            else:
                ops = self.core_context.searcher.operations()
            for op in ops:
                self._train_for_op(op, [
                    _TrainBoundary(_TrainBoundaryType.TRAIN,
                                   self.max_length if self.local_training else TrainUnit._from_searcher_unit(
                                       op.length, self.searcher_unit, self.global_batch_size)),
                    _TrainBoundary(_TrainBoundaryType.VALIDATE, self.validation_period),
                    _TrainBoundary(_TrainBoundaryType.CHECKPOINT, self.checkpoint_period),
                    _TrainBoundary(_TrainBoundaryType.REPORT, self.reporting_period),
                ])
                if self.test_mode:
                    break
        except ShouldExit as e:
            if not e.skip_exit_checkpoint and not self._checkpoint_is_current():
                self._checkpoint(already_exiting=True)
        except core.InvalidHP:
            if not self._checkpoint_is_current():
                self._checkpoint(already_exiting=True)
            raise


def _repeat(loader: Any, skip: int) -> Iterator:
    n = 0
    while True:
        for b in loader:
            if n < skip:
                n += 1
                continue
            yield b
