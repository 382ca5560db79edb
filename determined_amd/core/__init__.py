"""Core API: ``with core.init() as core_context: ...`` (reference ``harness/determined/core``)."""

from determined_amd.core._distributed import (
    DistributedContext,
    DummyDistributedContext,
    _run_on_rank_0_and_broadcast,
)
from determined_amd.core._checkpoint import CheckpointContext, DownloadMode, DummyCheckpointContext, merge_metadata
from determined_amd.core._train import TrainContext, DummyTrainContext, EarlyExitReason
from determined_amd.core._searcher import (
    DummySearcherContext,
    DummySearcherOperation,
    SearcherContext,
    SearcherMode,
    SearcherOperation,
    Unit,
    _parse_searcher_units,
)
from determined_amd.core._preempt import DummyPreemptContext, PreemptContext, PreemptMode
from determined_amd.core._profiler import DummyProfilerContext, ProfilerContext
from determined_amd.core._experimental import DummyExperimentalCoreContext, ExperimentalCoreContext
from determined_amd.core._context import Context, InvalidHP, init, _dummy_init
from determined_amd.core._tensorboard_mode import TensorboardMode
from determined_amd.core._heartbeat import UnmanagedTrialHeartbeat
