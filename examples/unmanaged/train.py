"""Unmanaged (Core API v2) training: the script runs wherever you start it -- no agent, no
scheduling -- and only *reports* to the master: an experiment + trial are created on first
``init`` and metrics / checkpoints appear in ``det experiment describe`` like any managed run
(reference: ``examples/features/unmanaged/1_singleton.py``, ``2_checkpoints.py``).

    DET_MASTER=http://127.0.0.1:8080 python train.py
"""

import os
import tempfile

from determined_amd.experimental import core_v2


def main() -> None:
    storage = os.environ.get("DET_UNMANAGED_STORAGE") or tempfile.mkdtemp(prefix="unmanaged-ckpt-")
    core_v2.init(
        defaults=core_v2.DefaultConfig(name="unmanaged-example", hparams={"lr": 0.1},
                                       checkpoint_storage={"type": "shared_fs", "host_path": storage}),
        unmanaged=core_v2.UnmanagedConfig(external_experiment_id=os.environ.get("EXTERNAL_EXP_ID", "unmanaged-ex"),
                                          external_trial_id=os.environ.get("EXTERNAL_TRIAL_ID", "trial-0")),
    )
    x = 1.0
    for step in range(1, 21):
        x *= 1.0 - core_v2.info.trial.hparams["lr"]
        core_v2.train.report_training_metrics(steps_completed=step, metrics={"loss": x})
        if step % 10 == 0:
            core_v2.train.report_validation_metrics(steps_completed=step, metrics={"validation_loss": x})
            with core_v2.checkpoint.store_path({"steps_completed": step}) as (path, uuid):
                (path / "state.txt").write_text(str(x))
    print(f"unmanaged trial {core_v2.info.trial.trial_id} of experiment {core_v2.info.trial.experiment_id} done")
    core_v2.close()


if __name__ == "__main__":
    main()
