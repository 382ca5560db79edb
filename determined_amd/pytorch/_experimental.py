"""``PyTorchTrialContext.experimental`` (reference: ``harness/determined/pytorch/_experimental.py``).

Three switches a trial flips in its ``__init__``:

* ``use_amp()`` -- automatic mixed precision for the simple cases: the wrapped models' forward
  runs under autocast, ``context.backward`` scales the loss, ``step_optimizer`` unscales before
  clipping and steps through the scaler, and the controller calls ``scaler.update()`` once per
  optimizer step (reference ``_pytorch_context.py:308,786,886`` / ``_pytorch_trial.py:857``).
  On a GPU the scaler is :class:`determined_amd.ops.DeviceGradScaler` (scale, unscale, inf check
  and skip stay on the device; with the fused optimizers the unscale happens inside the update
  kernel) and autocast runs fp16 -- the dtype loss scaling exists for.  On the CPU autocast runs
  bf16 and the scaler is disabled (bf16 needs no loss scaling).
* ``disable_dataset_reproducibility_checks()`` -- allow a plain ``torch.utils.data.DataLoader``
  from ``build_{training,validation}_data_loader`` (otherwise the controller requires
  ``determined_amd.pytorch.DataLoader``, whose samplers make shuffling, resumption and sharding
  reproducible).
* ``disable_auto_to_device()`` -- the controller stops moving batches to the device; the trial
  calls ``context.to_device`` on what it wants moved.
"""

import logging
from typing import Any

logger = logging.getLogger("determined_amd.pytorch")


class PyTorchExperimentalContext:
    def __init__(self, parent: Any) -> None:
        self._parent = parent
        self._auto_amp = False
        self._data_repro_checks_disabled = False
        self._auto_to_device = True

    def use_amp(self) -> None:
        """Automatic mixed precision with a default dynamic loss scaler (do not also call
        ``wrap_scaler``).  Call before ``wrap_model``."""
        from determined_amd.ops.scaler import DeviceGradScaler

        on_gpu = self._parent.device.type == "cuda"
        self._parent.wrap_scaler(DeviceGradScaler(enabled=on_gpu))
        self._auto_amp = True

    def disable_dataset_reproducibility_checks(self) -> None:
        self._data_repro_checks_disabled = True
        logger.info("disabled dataset reproducibility checks")

    def disable_auto_to_device(self) -> None:
        self._auto_to_device = False
        logger.info("disabled automatically moving data to device")
