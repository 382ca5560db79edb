"""Model hub adapters (reference: ``model_hub/``).  ``huggingface`` is available; the
``mmdetection`` adapter needs mmcv/mmdet, which are not in the ROCm image (gated)."""

from determined_amd.model_hub import utils
