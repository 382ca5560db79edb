"""PyTorch training API (reference: ``harness/determined/pytorch``)."""

from determined_amd.pytorch import samplers
from determined_amd.pytorch._data import DataLoader, TorchData, adapt_batch_sampler, data_length, to_device
from determined_amd.pytorch._callback import PyTorchCallback
from determined_amd.pytorch._lr_scheduler import LRScheduler
from determined_amd.pytorch._reducer import MetricReducer, Reducer, _PyTorchReducerContext, _SimpleReducer
from determined_amd.pytorch._context import PyTorchTrialContext
from determined_amd.pytorch._experimental import PyTorchExperimentalContext
from determined_amd.pytorch._trial import (
    Batch,
    Epoch,
    PyTorchTrial,
    TrainUnit,
    _PyTorchTrialController,
    _TrainBoundary,
    _TrainBoundaryType,
    _TrialState,
)
from determined_amd.pytorch._load import CheckpointLoadContext, load_trial_from_checkpoint_path
from determined_amd.pytorch._trainer import Trainer, init
