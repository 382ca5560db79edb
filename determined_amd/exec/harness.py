"""Trial-class entrypoint: ``python -m determined_amd.exec.harness model_def:MyTrial``
(reference: ``harness/determined/exec/harness.py``).

Loads the trial class from the model definition directory and runs it under ``pytorch.init()`` +
``Trainer.fit()`` (or the DeepSpeed-style ZeRO trial under its own controller).
"""

import faulthandler
import importlib
import logging
import os
import sys


def load_trial_class(entrypoint: str):
    module, _, qual = entrypoint.partition(":")
    if not qual:
        raise ValueError(f"entrypoint must look like 'module:TrialClass', got {entrypoint!r}")
    sys.path.insert(0, os.getcwd())
    obj = importlib.import_module(module)
    for part in qual.split("."):
        obj = getattr(obj, part)
    return obj


def main(entrypoint: str) -> int:
    from determined_amd import core, get_cluster_info, pytorch

    logging.basicConfig(level=logging.INFO, format="%(levelname)s: [%(process)s] %(name)s: %(message)s")
    if os.environ.get("DET_DEBUG") == "1":
        faulthandler.dump_traceback_later(30, repeat=True)
    info = get_cluster_info()
    assert info is not None and info.task_type == "TRIAL", "must be run on-cluster as a TRIAL task"
    trial_cls = load_trial_class(entrypoint)
    from determined_amd.pytorch.deepspeed import DeepSpeedTrial

    if isinstance(trial_cls, type) and issubclass(trial_cls, DeepSpeedTrial):
        from determined_amd.pytorch.deepspeed import run_deepspeed_trial

        return run_deepspeed_trial(trial_cls, info)
    if not (isinstance(trial_cls, type) and issubclass(trial_cls, pytorch.PyTorchTrial)):
        raise TypeError(f"{entrypoint} is not a PyTorchTrial subclass")
    try:
        with pytorch.init() as ctx:
            trial = trial_cls(ctx)
            pytorch.Trainer(trial, ctx).fit()
    except core.InvalidHP:
        return 0
    return 0


if __name__ == "__main__":
    if len(sys.argv) != 2:
        print("usage: python -m determined_amd.exec.harness module:TrialClass", file=sys.stderr)
        sys.exit(2)
    sys.exit(main(sys.argv[1]))
