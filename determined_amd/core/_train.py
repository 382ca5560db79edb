"""TrainContext: metric reporting (reference: ``harness/determined/core/_train.py``)."""

import enum
import logging
import math
import pathlib
from typing import Any, Callable, Dict, List, Optional

from determined_amd.common.api import NotFoundException

logger = logging.getLogger("determined_amd.core")

TRAINING = "training"
VALIDATION = "validation"


class EarlyExitReason(enum.Enum):
    INVALID_HP = "EXITED_REASON_INVALID_HP"
    USER_REQUESTED_STOP = "EXITED_REASON_USER_REQUESTED_STOP"


def _to_reportable(metrics: Dict[str, Any]) -> Dict[str, Any]:
    out = {}
    for k, v in metrics.items():
        if v is None:
            raise RuntimeError(f"metric {k!r} has no value (None)")
        if isinstance(v, (bytes, bytearray)):
            logger.warning(f"removing non-serializable metric {k}")
            continue
        if hasattr(v, "item") and getattr(v, "ndim", 0) == 0:
            v = v.item()
        elif hasattr(v, "tolist"):
            v = v.tolist()
        if isinstance(v, float) and not math.isfinite(v):
            v = str(v)  # JSON has no NaN/inf; the master stores the string form
        out[k] = v
    return out


class TrainContext:
    def __init__(self, session: Any, trial_id: int, run_id: int, exp_id: int, distributed: Any,
                 tensorboard_manager: Any = None, tbd_writer: Any = None) -> None:
        self._session = session
        self._trial_id = trial_id
        self._run_id = run_id
        self._exp_id = exp_id
        self._dist = distributed
        self._tensorboard_manager = tensorboard_manager
        self._tbd_writer = tbd_writer

    def set_status(self, status: str) -> None:
        self._session.post(f"/api/v1/trials/{self._trial_id}/runner/metadata", {"state": status})

    def _report_trial_metrics(self, group: str, steps_completed: int, metrics: Dict[str, Any],
                              batch_metrics: Optional[List[Dict[str, Any]]] = None) -> None:
        if "." in group:
            raise ValueError("metric group names cannot contain '.'")
        body = {
            "group": group,
            "steps_completed": int(steps_completed),
            "trial_run_id": self._run_id,
            "metrics": _to_reportable(metrics),
            "batch_metrics": [_to_reportable(b) for b in batch_metrics] if batch_metrics else None,
        }
        self._session.post(f"/api/v1/trials/{self._trial_id}/metrics", body)
        if self._tbd_writer is not None:
            self._tbd_writer.write(group, steps_completed, metrics)

    def report_training_metrics(self, steps_completed: int, metrics: Dict[str, Any],
                                batch_metrics: Optional[List[Dict[str, Any]]] = None) -> None:
        logger.info(f"report_training_metrics(steps_completed={steps_completed}, metrics={metrics})")
        self._report_trial_metrics(TRAINING, steps_completed, metrics, batch_metrics)

    def report_validation_metrics(self, steps_completed: int, metrics: Dict[str, Any]) -> None:
        logger.info(f"report_validation_metrics(steps_completed={steps_completed}, metrics={metrics})")
        self._report_trial_metrics(VALIDATION, steps_completed, metrics)

    def report_metrics(self, group: str, steps_completed: int, metrics: Dict[str, Any]) -> None:
        self._report_trial_metrics(group, steps_completed, metrics)

    def report_early_exit(self, reason: EarlyExitReason) -> None:
        self._session.post(f"/api/v1/trials/{self._trial_id}/early_exit", {"reason": EarlyExitReason(reason).value})

    def get_experiment_best_validation(self) -> Optional[float]:
        try:
            r = self._session.get(f"/api/v1/experiments/{self._exp_id}/searcher/best_searcher_validation_metric")
        except NotFoundException:
            return None
        return None if r is None or r.get("metric") is None else float(r["metric"])

    def get_tensorboard_path(self) -> pathlib.Path:
        if self._tensorboard_manager is None:
            raise ValueError("no tensorboard manager")
        return self._tensorboard_manager.base_path

    def upload_tensorboard_files(self, selector: Callable[[pathlib.Path], bool] = lambda _: True,
                                 mangler: Callable[[pathlib.Path, int], pathlib.Path] = lambda p, __: p) -> None:
        if self._tensorboard_manager is not None:
            self._tensorboard_manager.sync(selector, mangler, self._dist.rank)

    def _get_last_validation(self) -> Optional[int]:
        r = self._session.get(f"/api/v1/trials/{self._trial_id}")
        val = (r.get("trial") or {}).get("latest_validation") or {}
        return val.get("steps_completed")


class DummyTrainContext(TrainContext):
    def __init__(self, tensorboard_path: Optional[pathlib.Path] = None) -> None:
        self._tbd_directory = tensorboard_path
        self._tbd_writer = None
        self._tensorboard_manager = None
        self.reported: List[Dict[str, Any]] = []

    def set_status(self, status: str) -> None:
        logger.info(f"status: {status}")

    def _report_trial_metrics(self, group, steps_completed, metrics, batch_metrics=None) -> None:
        self.reported.append({"group": group, "steps_completed": steps_completed,
                              "metrics": _to_reportable(metrics)})

    def report_early_exit(self, reason: EarlyExitReason) -> None:
        logger.info(f"report_early_exit({reason})")

    def get_experiment_best_validation(self) -> Optional[float]:
        return None

    def get_tensorboard_path(self) -> pathlib.Path:
        return self._tbd_directory  # type: ignore

    def upload_tensorboard_files(self, selector=lambda _: True, mangler=lambda p, __: p) -> None:
        pass

    def _get_last_validation(self) -> Optional[int]:
        return None
