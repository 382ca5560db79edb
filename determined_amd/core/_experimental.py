"""``core_context.experimental`` (reference: ``harness/determined/core/_experimental.py``): link
the running task to the checkpoint / model version it uses (batch inference), so the metrics the
task reports show up under ``Checkpoint.get_metrics()`` / ``ModelVersion.get_metrics()``."""

import logging
from typing import Any

logger = logging.getLogger("determined_amd.core")


class ExperimentalCoreContext:
    def __init__(self, session: Any, trial_id: int) -> None:
        self._session = session
        self._trial_id = trial_id

    def _report(self, checkpoint_uuid: str, model_id: Any = None, model_version: Any = None) -> None:
        self._session.post("/api/v1/trial-source-info", {"trial_source_info": {
            "trial_id": self._trial_id, "checkpoint_uuid": checkpoint_uuid,
            "trial_source_info_type": "INFERENCE", "model_id": model_id, "model_version": model_version}})

    def report_task_using_checkpoint(self, checkpoint: Any) -> None:
        """Associate ``checkpoint`` (an SDK ``Checkpoint`` or a uuid) with this task."""
        self._report(getattr(checkpoint, "uuid", checkpoint))

    def report_task_using_model_version(self, model_version: Any) -> None:
        """Associate ``model_version`` (an SDK ``ModelVersion``) and its checkpoint with this task."""
        ck = model_version.checkpoint
        mid = getattr(model_version, "model_id", None)
        if mid is None:
            mid = self._session.get(f"/api/v1/models/{model_version.model_name}")["model"]["id"]
        self._report(getattr(ck, "uuid", ck), int(mid), int(model_version.model_version))


class DummyExperimentalCoreContext(ExperimentalCoreContext):
    """Off-cluster: nothing to link (the reference's dummy is a no-op too)."""

    def __init__(self) -> None:
        super().__init__(None, -1)

    def _report(self, checkpoint_uuid: str, model_id: Any = None, model_version: Any = None) -> None:
        logger.info("off-cluster: not linking this task to checkpoint %s", checkpoint_uuid)
