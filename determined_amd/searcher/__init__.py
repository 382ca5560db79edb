"""Hyperparameter search: native search methods + the custom-searcher API
(reference: ``master/pkg/searcher`` and ``harness/determined/searcher``)."""

from determined_amd.searcher._native_searcher import Searcher, decode_sample, flatten_hparams, simulate
from determined_amd.searcher._custom import (
    Close,
    Create,
    ExitedReason,
    LocalSearchRunner,
    Operation,
    Progress,
    RemoteSearchRunner,
    SearchMethod,
    SearchRunner,
    SearcherState,
    Shutdown,
    ValidateAfter,
)
