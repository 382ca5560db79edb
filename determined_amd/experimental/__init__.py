"""Experimental APIs (reference: ``harness/determined/experimental``): the SDK ``client``,
unmanaged Core API v2 (``core_v2``)."""

from determined_amd.experimental import client
from determined_amd.experimental import core_v2
from determined_amd.experimental.client import (
    Checkpoint,
    Experiment,
    Model,
    ModelVersion,
    Project,
    Trial,
    User,
    Workspace,
)
from determined_amd.experimental.determined import (
    Determined,
    ResourcePool,
    TrainingMetrics,
    TrialMetrics,
    ValidationMetrics,
    test_one_batch,
)
