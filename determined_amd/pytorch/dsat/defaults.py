"""DeepSpeed-autotune (dsat) defaults (reference: ``harness/determined/pytorch/dsat/defaults.py``)."""

ALL_SEARCH_METHOD_NAMES = ["binary", "random", "_test"]
USE_DSAT_MODE_KEY = "_dsat_mode"
CONFIG_KEY = "deepspeed_config"
OVERWRITE_KEY = "overwrite_deepspeed_args"

SMALLER_IS_BETTER_METRICS = ["latency"]
LARGER_IS_BETTER_METRICS = ["throughput"]

AUTOTUNING_ARG_DEFAULTS = {
    "max_trials": 32,
    "max_concurrent_trials": 8,
    "zero_stages": [1, 2, 3],
    "start_profile_step": 3,
    "end_profile_step": 5,
    "metric": "throughput",
    "random_seed": 42,
    "max_mbs": 128,
    "min_mbs": 1,
    "run_full_experiment": False,
}
