"""DeepSpeedTrialContext (reference: ``harness/determined/pytorch/deepspeed/_deepspeed_context.py``).

Engines come from ``determined_amd.parallel.zero.initialize`` (our ZeRO engine) instead of
``deepspeed.initialize``; everything the trial sees (``wrap_model_engine``, ``set_mpu``,
``disable_auto_grad_accumulation``, ``train_micro_batch_size_per_gpu``,
``num_micro_batches_per_slot``, tensorboard, reducers, hparams) matches the reference.
"""

import copy
import json
import logging
import os
from typing import Any, Dict, Union

from determined_amd.pytorch._context import PyTorchTrialContext
from determined_amd.pytorch.deepspeed._mpu import ModelParallelUnit, make_data_parallel_mpu

logger = logging.getLogger("determined_amd.pytorch.deepspeed")


class InvalidExperimentException(Exception):
    pass


def _merge(base: Dict[str, Any], src: Dict[str, Any]) -> Dict[str, Any]:
    out = copy.deepcopy(base)
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def overwrite_deepspeed_config(base_ds_config: Union[str, os.PathLike, Dict[str, Any]],
                               source_ds_dict: Dict[str, Any]) -> Dict[str, Any]:
    """Recursively overwrite ``base_ds_config`` (dict or JSON path) with ``source_ds_dict``
    (reference ``_deepspeed_context.py:18``)."""
    if isinstance(base_ds_config, (str, os.PathLike)):
        def no_dupes(pairs):
            d: Dict[str, Any] = {}
            for k, v in pairs:
                if k in d:
                    raise ValueError(f"duplicate key {k!r} in DeepSpeed config")
                d[k] = v
            return d

        with open(base_ds_config) as f:
            base_ds_config = json.load(f, object_pairs_hook=no_dupes)
    elif not isinstance(base_ds_config, dict):
        raise TypeError("Expected string or dict for base_ds_config argument.")
    return _merge(base_ds_config, source_ds_dict or {})


class DeepSpeedTrialContext(PyTorchTrialContext):
    def __init__(self, *args: Any, **kwargs: Any) -> None:
        super().__init__(*args, **kwargs)
        self._mpu = make_data_parallel_mpu(self.distributed)
        self._called_set_mpu = False
        self._train_micro_batch_size_per_gpu = None
        self._num_micro_batches_per_slot = None
        self._use_pipeline_parallel = False
        self._data_repro_checks_disabled = False
        self._manual_grad_accumulation = False
        self._check_experiment_config_optimizations()

    def _check_experiment_config_optimizations(self) -> None:
        opt = (self._exp_conf or {}).get("optimizations", {}) or {}
        if opt.get("mixed_precision", "O0") != "O0":
            raise InvalidExperimentException(
                "Mixed precision is specified through the deepspeed config instead of the experiment config.")
        if int(opt.get("aggregation_frequency", 1)) > 1:
            raise InvalidExperimentException(
                "Gradient aggregation is specified through the deepspeed config instead of the experiment config.")
        for field, default in {"average_aggregated_gradients": True, "gradient_compression": False,
                               "tensor_fusion_threshold": 64, "tensor_fusion_cycle_time": 5,
                               "autotune_tensor_fusion": False}.items():
            if opt.get(field, default) != default:
                logger.warning("%s=%s ignored since the setting does not apply to DeepSpeedTrial.", field,
                               opt.get(field))

    # -- engines -------------------------------------------------------------------------------
    def wrap_model_engine(self, model: Any) -> Any:
        """Register a ZeRO model engine (first one defines micro-batch size and accumulation)."""
        model = model.to(self.device)
        if getattr(model, "is_pipe_parallel", False):
            self._use_pipeline_parallel = True
            if not self.models and hasattr(model, "mpu"):
                self._mpu = model.mpu
        if not self.models:
            self._train_micro_batch_size_per_gpu = int(model.train_micro_batch_size_per_gpu())
            self._num_micro_batches_per_slot = int(model.gradient_accumulation_steps())
        elif model.train_micro_batch_size_per_gpu() != self._train_micro_batch_size_per_gpu:
            logger.warning("Train micro batch size for wrapped model engine %d does not match that for the first "
                           "wrapped engine.", len(self.models) + 1)
        self.models.append(model)
        return model

    def set_mpu(self, mpu: ModelParallelUnit) -> None:
        if not self.models:
            raise InvalidExperimentException("Please call `wrap_model_engine` before setting the mpu.")
        if self._called_set_mpu:
            raise InvalidExperimentException("Only one MPU can be passed to DeepSpeedTrialContext.")
        avg = bool((self._exp_conf or {}).get("optimizations", {}).get("average_training_metrics", True))
        if self.distributed.rank == 0 and not mpu.should_report_metrics and not avg:
            raise InvalidExperimentException(
                "Please set optimizations.average_training_metrics in the experiment config to true so that "
                "metrics will exist on the chief for report to the master.")
        self._called_set_mpu = True
        self._mpu = mpu

    def disable_auto_grad_accumulation(self) -> None:
        self._manual_grad_accumulation = True

    def disable_dataset_reproducibility_checks(self) -> None:
        self._data_repro_checks_disabled = True

    @property
    def use_pipeline_parallel(self) -> bool:
        return self._use_pipeline_parallel

    @property
    def train_micro_batch_size_per_gpu(self) -> int:
        if self._train_micro_batch_size_per_gpu is None:
            raise InvalidExperimentException("Please call wrap_model_engine before accessing train_micro_batch_size.")
        return self._train_micro_batch_size_per_gpu

    @property
    def num_micro_batches_per_slot(self) -> int:
        if self._num_micro_batches_per_slot is None:
            raise InvalidExperimentException(
                "Please call wrap_model_engine before accessing num_micro_batches_per_slot.")
        return self._num_micro_batches_per_slot

    def get_global_batch_size(self) -> int:
        if self.models:
            return int(self.models[0].train_batch_size())
        return super().get_global_batch_size()

    # -- PyTorchTrial-only APIs do not apply ------------------------------------------------------
    def wrap_model(self, model: Any) -> Any:  # type: ignore[override]
        raise InvalidExperimentException("DeepSpeedTrial: build an engine with zero.initialize() and call "
                                         "wrap_model_engine() instead of wrap_model()")

    def wrap_optimizer(self, *a: Any, **k: Any) -> Any:  # type: ignore[override]
        raise InvalidExperimentException("DeepSpeedTrial: the optimizer belongs to the model engine")

    def backward(self, *a: Any, **k: Any) -> None:  # type: ignore[override]
        raise InvalidExperimentException("DeepSpeedTrial: call model_engine.backward(loss)")

    def step_optimizer(self, *a: Any, **k: Any) -> None:  # type: ignore[override]
        raise InvalidExperimentException("DeepSpeedTrial: call model_engine.step()")
