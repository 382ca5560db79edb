"""DeepSpeed autotuning ("dsat") for DeepSpeedTrial over the native ZeRO engine (reference:
``harness/determined/pytorch/dsat``).  See ``_search.py`` for the search methods and
``__main__.py`` for the ``python -m determined_amd.pytorch.dsat`` entry point."""

from determined_amd.pytorch.dsat import defaults
from determined_amd.pytorch.dsat._search import (
    METHODS,
    BaseDSATSearchMethod,
    BinarySearchDSATSearchMethod,
    Candidate,
    RandomDSATSearchMethod,
    TestDSATSearchMethod,
    candidate_hparams,
)
from determined_amd.pytorch.dsat._run import build_search_method, get_ds_config_from_hparams, run_autotuning
