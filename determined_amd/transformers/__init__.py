"""HuggingFace Transformers integration (reference: ``harness/determined/transformers``)."""

from determined_amd.transformers._hf_callback import (
    DetCallback,
    get_ds_config_path_from_args,
    get_metric_type,
)
from determined_amd.transformers._optim import fused_optimizer
from determined_amd.transformers._kernels import accelerate
