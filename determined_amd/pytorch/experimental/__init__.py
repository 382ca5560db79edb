"""Experimental PyTorch APIs (reference: ``harness/determined/pytorch/experimental``)."""

from determined_amd.pytorch.experimental._torch_batch_process import (
    TorchBatchProcessor,
    TorchBatchProcessorContext,
    torch_batch_process,
)
