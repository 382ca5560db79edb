"""DeepSpeedTrial and its controller (reference:
``harness/determined/pytorch/deepspeed/_deepspeed_trial.py``).

Semantics kept from the reference:

* ``train_batch(dataloader_iter, epoch_idx, batch_idx)`` receives the *iterator* of
  micro-batches; the controller calls it ``gradient_accumulation_steps`` times per batch
  (once when pipeline parallel or ``disable_auto_grad_accumulation()``) and checks that the
  engine took that many micro-steps (reference ``_train_for_step``, ``:364``);
* ``evaluate_batch(dataloader_iter, batch_idx)`` is called ``num_validation_batches`` times
  (minimum over ranks of the per-rank validation loader length);
* checkpoints: every rank writes ``det_state_dict_rank{r}.pth`` (RNG + callback state) and
  the trial's ``save`` (default: each engine's ``save_checkpoint(path, tag=f"model{i}")``,
  i.e. model weights from rank 0 plus one optimizer shard per rank) into ONE sharded
  checkpoint (``core.checkpoint.store_path(shard=True)``).

MI355X-native: the engine is ``determined_amd.parallel.zero.ZeroEngine`` (RCCL
reduce-scatter / all-gather, fused AdamW on shards); training metrics stay on the device
until the reporting period like the PyTorchTrial controller.
"""

import abc
import contextlib
import json
import logging
import os
import pathlib
from typing import Any, Dict, Iterator, List, Optional, Union

import torch

from determined_amd import core
from determined_amd.pytorch import _data
from determined_amd.pytorch._callback import PyTorchCallback
from determined_amd.pytorch._reducer import Reducer
from determined_amd.pytorch._trainer import Trainer, _init_context
from determined_amd.pytorch._trial import (
    CHECKPOINT_FORMAT,
    _PyTorchTrialController,
    _rng_state,
    _set_rng_state,
    _TrialState,
)
from determined_amd.pytorch.deepspeed._context import DeepSpeedTrialContext, InvalidExperimentException

logger = logging.getLogger("determined_amd.pytorch.deepspeed")


def _repro_error(name: str, obj: Any) -> str:
    return (f"{name}() returned {type(obj).__name__}, not determined_amd.pytorch.DataLoader; call "
            "context.disable_dataset_reproducibility_checks() to use an arbitrary loader (it must then repeat "
            "indefinitely and shard itself).")


class DeepSpeedTrialController(_PyTorchTrialController):
    def __init__(self, trial_inst: "DeepSpeedTrial", context: DeepSpeedTrialContext, **kw: Any) -> None:
        if not isinstance(trial_inst, DeepSpeedTrial):
            raise TypeError("DeepSpeedTrialController needs a DeepSpeedTrial")
        if not context.models:
            raise InvalidExperimentException("Must have at least one model engine. This might be caused by not "
                                             "wrapping your model with wrap_model_engine()")
        super().__init__(trial_inst, context, **kw)
        self.context: DeepSpeedTrialContext = context
        # DeepSpeed autotuning profiling run (``pytorch/dsat``): time a window of batches and
        # report throughput/latency instead of validating; OOM -> InvalidHP (early exit)
        self._dsat: Optional[Dict[str, Any]] = (context.get_hparams() or {}).get("_dsat_mode") or None
        self._dsat_t0: Optional[float] = None
        self._dsat_t1: Optional[float] = None

    # -- data ------------------------------------------------------------------------------------
    def _set_data_loaders(self) -> None:
        ctx = self.context
        mpu = ctx._mpu
        gas = ctx.num_micro_batches_per_slot
        skip = self.state.batches_trained * gas  # every batch consumes gas micro-batches per slot
        self.training_loader: Any = None
        self.validation_loader: Any = None
        n_train: Optional[int] = None
        n_val: Optional[int] = None
        if mpu.should_build_data_loader:
            tl = self.trial.build_training_data_loader()
            if isinstance(tl, _data.DataLoader):
                self.training_loader = tl.get_data_loader(repeat=True, skip=skip,
                                                          num_replicas=mpu.data_parallel_world_size,
                                                          rank=mpu.data_parallel_rank, seed=ctx.get_trial_seed())
                n_train = len(tl) // max(mpu.data_parallel_world_size, 1)
            else:
                if not ctx._data_repro_checks_disabled:
                    raise RuntimeError(_repro_error("build_training_data_loader", tl))
                logger.warning("Please make sure custom data loader repeats indefinitely.")
                self.training_loader = tl
                n_train = _data._dataset_len(tl)
            vl = self.trial.build_validation_data_loader()
            if isinstance(vl, _data.DataLoader):
                self.validation_loader = vl.get_data_loader(repeat=False, num_replicas=mpu.data_parallel_world_size,
                                                            rank=mpu.data_parallel_rank)
            elif vl is not None:
                if not ctx._data_repro_checks_disabled:
                    raise RuntimeError(_repro_error("build_validation_data_loader", vl))
                self.validation_loader = vl
            if self.validation_loader is not None:
                n_val = len(self.validation_loader)
                if ctx.use_pipeline_parallel:
                    n_val //= gas
        lens = [x for x in self.context.distributed.allgather(n_train) if x is not None]
        if lens and min(lens) < max(lens):
            logger.warning("Training data loader length inconsistent across ranks. Using the minimum.")
        ctx._epoch_len = max((min(lens) if lens else 1) // gas, 1)
        self._train_loader_len = ctx._epoch_len
        vlens = [x for x in self.context.distributed.allgather(n_val) if x is not None]
        if vlens and min(vlens) < max(vlens):
            logger.warning("Validation data loader length inconsistent across ranks. Using the minimum.")
        self.num_validation_batches = min(vlens) if vlens else 0
        self._val_shard = (1, 0)

    def _make_training_enumerator(self) -> Iterator:
        self.training_iterator = iter(self.training_loader) if self.training_loader is not None else None
        i = self.state.batches_trained
        while True:
            yield i, None
            i += 1

    # -- train -----------------------------------------------------------------------------------
    def _train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, Any]:
        if self._dsat is None:
            return self._train_batch_inner(batch, epoch_idx, batch_idx)
        import time

        start, end = int(self._dsat["start_profile_step"]), int(self._dsat["end_profile_step"])
        try:
            if batch_idx == start:
                self._sync_device()
                self._dsat_t0 = time.perf_counter()
            out = self._train_batch_inner(batch, epoch_idx, batch_idx)
            if batch_idx + 1 == end:
                self._sync_device()
                self._dsat_t1 = time.perf_counter()
            return out
        except torch.OutOfMemoryError as e:
            raise core.InvalidHP(f"dsat: out of memory at micro-batch "
                                 f"{self.context.train_micro_batch_size_per_gpu}: {e}") from None
        except RuntimeError as e:
            if "out of memory" in str(e).lower():
                raise core.InvalidHP(f"dsat: out of memory: {e}") from None
            raise

    def _sync_device(self) -> None:
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def _validate(self, op: Any = None) -> Dict[str, Any]:
        if self._dsat is None:
            return super()._validate(op)
        start, end = int(self._dsat["start_profile_step"]), int(self._dsat["end_profile_step"])
        if self._dsat_t0 is None or self._dsat_t1 is None or self.state.batches_trained < end:
            self.state.last_val = self.state.batches_trained
            return {}
        dt = max(self._dsat_t1 - self._dsat_t0, 1e-9)
        ctx = self.context
        samples = (end - start) * ctx.train_micro_batch_size_per_gpu * ctx.num_micro_batches_per_slot
        dts = [x for x in ctx.distributed.allgather(dt)]
        dt = max(dts)  # the slowest rank bounds the step
        metrics = {"throughput": samples / dt, "latency": dt / (end - start),
                   "train_micro_batch_size_per_gpu": ctx.train_micro_batch_size_per_gpu,
                   "zero_stage": int(getattr(ctx.models[0], "stage", -1))}
        self.state.last_val = self.state.batches_trained
        if self.is_chief:
            self.core_context.train.report_validation_metrics(self.state.batches_trained, metrics)
            if op is not None and not op._completed:
                op.report_completed(float(metrics[self._dsat.get("metric", "throughput")]))
        return metrics

    def _train_batch_inner(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, Any]:
        ctx = self.context
        calls = 1 if (ctx.use_pipeline_parallel or ctx._manual_grad_accumulation) else ctx.num_micro_batches_per_slot
        per_micro: List[Dict[str, Any]] = []
        for _ in range(calls):
            with contextlib.ExitStack() as st:
                if ctx.profiler is not None:
                    st.enter_context(ctx.profiler)
                out = self.trial.train_batch(self.training_iterator, epoch_idx, batch_idx)
                if ctx.profiler is not None:
                    ctx.profiler.step()
            if ctx._mpu.should_report_metrics:
                if isinstance(out, torch.Tensor):
                    out = {"loss": out}
                if not isinstance(out, dict):
                    raise InvalidExperimentException(
                        f"train_batch must return a dictionary mapping string names to Tensor metrics, got {type(out)}")
                per_micro.append({k: (v.detach() if isinstance(v, torch.Tensor) else v) for k, v in out.items()})
        model0 = ctx.models[0]
        if not ctx.use_pipeline_parallel and hasattr(model0, "micro_steps"):
            if model0.micro_steps % ctx.num_micro_batches_per_slot != 0:
                raise RuntimeError("did not train for gradient accumulation steps")
        if not per_micro:
            return {}
        if len(per_micro) == 1:
            return per_micro[0]
        merged: Dict[str, Any] = {}
        for k in per_micro[0]:
            vals = [m[k] for m in per_micro if k in m]
            if all(isinstance(v, torch.Tensor) and v.numel() == 1 for v in vals):
                merged[k] = torch.stack([v.float().reshape(()) for v in vals]).mean()
            elif all(isinstance(v, (int, float)) for v in vals):
                merged[k] = sum(vals) / len(vals)
            else:
                merged[k] = vals[-1]
        return merged

    # -- validate --------------------------------------------------------------------------------
    def _evaluate_batch_defined(self) -> bool:
        return True

    def _iter_eval_metrics(self) -> Iterator[Dict[str, Any]]:
        it = iter(self.validation_loader) if self.validation_loader is not None else None
        for idx in range(self.num_validation_batches):
            vm = self.trial.evaluate_batch(it, idx)
            if self.context._mpu.should_report_metrics:
                yield vm
            if self.test_mode:
                break

    # -- checkpoint ------------------------------------------------------------------------------
    def _checkpoint(self, already_exiting: bool) -> None:
        if self._dsat is not None:  # profiling runs never checkpoint
            self.state.last_ckpt = self.state.batches_trained
            return
        if self.is_chief:
            self.core_context.train.set_status("checkpointing")
        self.state.last_ckpt = self.state.batches_trained
        metadata = {"steps_completed": self.state.batches_trained, "framework": f"torch-{torch.__version__}",
                    "format": CHECKPOINT_FORMAT + "-deepspeed"}
        with self.core_context.checkpoint.store_path(metadata, shard=True) as (path, storage_id):
            self._save(path)
        if self.is_chief:
            for cb in self.callbacks.values():
                cb.on_checkpoint_upload_end(storage_id)

    def _save(self, path: pathlib.Path) -> None:
        dist = self.context.distributed
        path.mkdir(parents=True, exist_ok=True)
        ckpt: Dict[str, Any] = {"rng_state": _rng_state(),
                                "callbacks": {n: cb.state_dict() for n, cb in self.callbacks.items()}}
        for cb in self.callbacks.values():
            cb.on_checkpoint_save_start(ckpt)
        torch.save(ckpt, str(path / f"det_state_dict_rank{dist.rank}.pth"))
        if self.is_chief:
            with open(path / "trial_state.json", "w") as f:
                json.dump(self.state.to_dict(), f)
            cls = type(self.trial)
            try:
                exp_conf: Optional[Dict[str, Any]] = self.context.get_experiment_config()
                hparams: Optional[Dict[str, Any]] = self.context.get_hparams()
            except ValueError:
                exp_conf, hparams = None, None
            with open(path / "load_data.json", "w") as f:
                json.dump({"trial_type": "DeepSpeedTrial", "experiment_config": exp_conf, "hparams": hparams,
                           "trial_cls_spec": f"{cls.__module__}:{cls.__qualname__}", "is_trainer": True,
                           "format": CHECKPOINT_FORMAT + "-deepspeed"}, f, default=str)
            code_dir = os.environ.get("DET_MODEL_DEF_DIR")
            if code_dir and os.path.isdir(code_dir):
                import shutil

                shutil.copytree(code_dir, path / "code", dirs_exist_ok=True,
                                ignore=shutil.ignore_patterns("__pycache__", "*.pyc"))
        self.trial.save(self.context, path)
        for cb in self.callbacks.values():
            cb.on_checkpoint_end(str(path))
            cb.on_checkpoint_write_end(str(path))

    def _load(self, load_path: pathlib.Path) -> None:
        dist = self.context.distributed
        p = load_path / f"det_state_dict_rank{dist.rank}.pth"
        ckpt: Dict[str, Any] = {}
        if p.exists():
            ckpt = torch.load(str(p), map_location="cpu", weights_only=True)
        for cb in self.callbacks.values():
            cb.on_checkpoint_load_start(ckpt)
        self.trial.load(self.context, load_path)
        if "rng_state" in ckpt:
            _set_rng_state(ckpt["rng_state"])
        else:
            logger.warning("The checkpoint has no random state to restore.")
        for name, cb in self.callbacks.items():
            if name in ckpt.get("callbacks", {}):
                cb.load_state_dict(ckpt["callbacks"][name])
        ts = load_path / "trial_state.json"
        if ts.exists():
            st = json.loads(ts.read_text())
            self.state = _TrialState(**{k: v for k, v in st.items() if k in vars(_TrialState())})
            if self.state.trial_id != self.context.get_trial_id():
                self.state = _TrialState(trial_id=self.context.get_trial_id())
        else:
            self.state = _TrialState(trial_id=self.context.get_trial_id(), batches_trained=self.steps_completed)


class DeepSpeedTrial(metaclass=abc.ABCMeta):
    """User-facing trial for ZeRO-engine training (reference ``_deepspeed_trial.py:729``).

    .. code-block:: python

        class MyTrial(DeepSpeedTrial):
            def __init__(self, context):
                self.context = context
                model = build_model()
                ds_config = overwrite_deepspeed_config("ds_config.json",
                                                      context.get_hparam("overwrite_deepspeed_args"))
                engine, _, _, _ = zero.initialize(model=model, model_parameters=model.parameters(),
                                                  config=ds_config)
                self.model_engine = context.wrap_model_engine(engine)

            def train_batch(self, dataloader_iter, epoch_idx, batch_idx):
                batch = self.context.to_device(next(dataloader_iter))
                loss = self.model_engine(batch)
                self.model_engine.backward(loss)
                self.model_engine.step()
                return {"loss": loss}
    """

    trial_controller_class = DeepSpeedTrialController
    trial_context_class = DeepSpeedTrialContext

    def __init__(self, context: DeepSpeedTrialContext) -> None:
        pass

    @abc.abstractmethod
    def train_batch(self, dataloader_iter: Optional[Iterator[Any]], epoch_idx: int, batch_idx: int
                    ) -> Union[torch.Tensor, Dict[str, Any]]:
        pass

    @abc.abstractmethod
    def build_training_data_loader(self) -> Any:
        pass

    @abc.abstractmethod
    def build_validation_data_loader(self) -> Any:
        pass

    def build_callbacks(self) -> Dict[str, PyTorchCallback]:
        return {}

    @abc.abstractmethod
    def evaluate_batch(self, dataloader_iter: Optional[Iterator[Any]], batch_idx: int) -> Dict[str, Any]:
        pass

    def evaluation_reducer(self) -> Union[Reducer, Dict[str, Reducer]]:
        return Reducer.AVG

    def save(self, context: DeepSpeedTrialContext, path: pathlib.Path) -> None:
        """Default: every engine writes ``path/model{i}/`` (weights from rank 0, one optimizer shard
        per rank).  Override for custom layouts."""
        for i, m in enumerate(context.models):
            m.save_checkpoint(str(path), tag=f"model{i}", save_latest=False)

    def load(self, context: DeepSpeedTrialContext, load_dir: pathlib.Path) -> None:
        for i, m in enumerate(context.models):
            p, _ = m.load_checkpoint(str(load_dir), tag=f"model{i}")
            if p is None:
                raise RuntimeError(f"DeepSpeed checkpoint for engine {i} not found in {load_dir}")


@contextlib.contextmanager
def init(*, hparams: Optional[Dict[str, Any]] = None, exp_conf: Optional[Dict[str, Any]] = None,
         distributed: Optional[core.DistributedContext] = None, enable_tensorboard_logging: bool = True,
         checkpoint_storage: Any = None) -> Iterator[DeepSpeedTrialContext]:
    """Like ``pytorch.init()`` but yields a DeepSpeedTrialContext (local or on-cluster)."""
    with _init_context(DeepSpeedTrialContext, hparams=hparams, exp_conf=exp_conf, distributed=distributed,
                       aggregation_frequency=1, enable_tensorboard_logging=enable_tensorboard_logging,
                       checkpoint_storage=checkpoint_storage, ddp_bucket_mb=16.0) as ctx:
        yield ctx


def run_deepspeed_trial(trial_cls: Any, info: Any = None) -> int:
    """Entry used by ``exec.harness`` for DeepSpeedTrial subclasses (on-cluster)."""
    try:
        with init() as ctx:
            trial = trial_cls(ctx)
            Trainer(trial, ctx).fit()
    except core.InvalidHP:
        return 0
    return 0
