"""DeepSpeedTrial API over the native ZeRO engine (filled in by _trial.py)."""

from determined_amd.pytorch.deepspeed._trial import DeepSpeedTrial, DeepSpeedTrialContext, run_deepspeed_trial
