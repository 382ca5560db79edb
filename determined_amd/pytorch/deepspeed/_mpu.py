"""Model-parallel unit: which data-parallel replica a rank is and what it is responsible for
(reference: ``harness/determined/pytorch/deepspeed/_mpu.py``)."""

import dataclasses
from typing import Any


@dataclasses.dataclass
class ModelParallelUnit:
    data_parallel_rank: int
    data_parallel_world_size: int
    # the rank returns metrics from train/evaluate (e.g. last pipeline / tensor-parallel rank 0)
    should_report_metrics: bool
    # the rank needs a data loader (ranks in the middle of a pipeline do not)
    should_build_data_loader: bool


def make_data_parallel_mpu(dist_context: Any) -> ModelParallelUnit:
    return ModelParallelUnit(data_parallel_rank=dist_context.get_rank(),
                             data_parallel_world_size=dist_context.get_size(),
                             should_report_metrics=True, should_build_data_loader=True)


def make_tensor_parallel_mpu(dist_context: Any, tp_size: int) -> ModelParallelUnit:
    """Consecutive ranks form a tensor-parallel group; every TP rank sees the same batch."""
    rank, size = dist_context.get_rank(), dist_context.get_size()
    if size % tp_size:
        raise ValueError(f"world size {size} is not divisible by tensor-parallel size {tp_size}")
    return ModelParallelUnit(data_parallel_rank=rank // tp_size, data_parallel_world_size=size // tp_size,
                             should_report_metrics=True, should_build_data_loader=True)
