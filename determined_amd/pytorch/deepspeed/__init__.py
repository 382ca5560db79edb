"""DeepSpeedTrial API over the native ZeRO engine (reference:
``harness/determined/pytorch/deepspeed/__init__.py``).

``initialize`` is ``determined_amd.parallel.zero.initialize`` (the ``deepspeed.initialize``
equivalent) re-exported for convenience.
"""

from determined_amd.parallel.zero import DeepSpeedConfig, ZeroEngine, initialize
from determined_amd.pytorch.deepspeed._mpu import (
    ModelParallelUnit,
    make_data_parallel_mpu,
    make_tensor_parallel_mpu,
)
from determined_amd.pytorch.deepspeed._context import (
    DeepSpeedTrialContext,
    InvalidExperimentException,
    overwrite_deepspeed_config,
)
from determined_amd.pytorch.deepspeed._trial import (
    DeepSpeedTrial,
    DeepSpeedTrialController,
    init,
    run_deepspeed_trial,
)
