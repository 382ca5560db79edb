"""Custom search methods (reference: ``harness/determined/searcher/_search_method.py``,
``_search_runner.py``, ``_remote_search_runner.py``).

A user ``SearchMethod`` reacts to searcher events (trial created / validation completed / trial
closed / exited early) with operations (Create / ValidateAfter / Close / Shutdown / Progress).
A ``SearchRunner`` creates an experiment with ``searcher.name: custom`` on the master, then
long-polls its event queue, calls the method, and posts the operations back.
"""

import abc
import base64
import enum
import io
import json
import logging
import pathlib
import tarfile
import time
import uuid
from typing import Any, Dict, List, Optional, Set, Tuple

logger = logging.getLogger("determined_amd.searcher")


class ExitedReason(enum.Enum):
    ERRORED = "errored"
    USER_CANCELED = "user_canceled"
    INVALID_HP = "invalid_hp"
    INIT_INVALID_HP = "init_invalid_hp"
    USER_REQUESTED_STOP = "user_requested_stop"


class SearcherState:
    def __init__(self) -> None:
        self.failures: Set[uuid.UUID] = set()
        self.trial_progress: Dict[uuid.UUID, float] = {}
        self.trials_closed: Set[uuid.UUID] = set()
        self.trials_created: Set[uuid.UUID] = set()
        self.experiment_completed = False
        self.experiment_failed = False
        self.last_event_id = 0

    def to_dict(self) -> Dict[str, Any]:
        return {"failures": [str(x) for x in self.failures],
                "trial_progress": {str(k): v for k, v in self.trial_progress.items()},
                "trials_closed": [str(x) for x in self.trials_closed],
                "trials_created": [str(x) for x in self.trials_created],
                "experiment_completed": self.experiment_completed, "experiment_failed": self.experiment_failed,
                "last_event_id": self.last_event_id}

    def from_dict(self, d: Dict[str, Any]) -> None:
        self.failures = {uuid.UUID(x) for x in d["failures"]}
        self.trial_progress = {uuid.UUID(k): v for k, v in d["trial_progress"].items()}
        self.trials_closed = {uuid.UUID(x) for x in d["trials_closed"]}
        self.trials_created = {uuid.UUID(x) for x in d["trials_created"]}
        self.experiment_completed = d["experiment_completed"]
        self.experiment_failed = d.get("experiment_failed", False)
        self.last_event_id = d["last_event_id"]


class Operation(metaclass=abc.ABCMeta):
    @abc.abstractmethod
    def to_wire(self) -> Dict[str, Any]:
        pass


class ValidateAfter(Operation):
    def __init__(self, request_id: uuid.UUID, length: int) -> None:
        self.request_id = request_id
        self.length = int(length)

    def to_wire(self) -> Dict[str, Any]:
        return {"type": "validate_after", "request_id": str(self.request_id), "length": self.length}


class Close(Operation):
    def __init__(self, request_id: uuid.UUID) -> None:
        self.request_id = request_id

    def to_wire(self) -> Dict[str, Any]:
        return {"type": "close", "request_id": str(self.request_id)}


class Progress(Operation):
    def __init__(self, progress: float) -> None:
        self.progress = float(progress)

    def to_wire(self) -> Dict[str, Any]:
        return {"type": "progress", "progress": self.progress}


class Shutdown(Operation):
    def __init__(self, cancel: bool = False, failure: bool = False) -> None:
        self.cancel = cancel
        self.failure = failure

    def to_wire(self) -> Dict[str, Any]:
        return {"type": "shutdown", "cancel": self.cancel, "failure": self.failure}


class Create(Operation):
    def __init__(self, request_id: uuid.UUID, hparams: Dict[str, Any], checkpoint: Optional[str] = None) -> None:
        self.request_id = request_id
        self.hparams = hparams
        self.checkpoint = checkpoint

    def to_wire(self) -> Dict[str, Any]:
        return {"type": "create", "request_id": str(self.request_id), "hparams": self.hparams,
                "checkpoint": self.checkpoint}


class SearchMethod:
    @abc.abstractmethod
    def initial_operations(self, searcher_state: SearcherState) -> List[Operation]:
        pass

    @abc.abstractmethod
    def on_trial_created(self, searcher_state: SearcherState, request_id: uuid.UUID) -> List[Operation]:
        pass

    @abc.abstractmethod
    def on_validation_completed(self, searcher_state: SearcherState, request_id: uuid.UUID, metric: Any,
                                train_length: int) -> List[Operation]:
        pass

    @abc.abstractmethod
    def on_trial_closed(self, searcher_state: SearcherState, request_id: uuid.UUID) -> List[Operation]:
        pass

    @abc.abstractmethod
    def progress(self, searcher_state: SearcherState) -> float:
        pass

    @abc.abstractmethod
    def on_trial_exited_early(self, searcher_state: SearcherState, request_id: uuid.UUID,
                              exited_reason: ExitedReason) -> List[Operation]:
        pass

    def save_method_state(self, path: pathlib.Path) -> None:
        pass

    def load_method_state(self, path: pathlib.Path) -> None:
        pass

    def save(self, searcher_state: SearcherState, path: pathlib.Path, *, experiment_id: int) -> None:
        path.mkdir(parents=True, exist_ok=True)
        (path / "searcher_state.json").write_text(json.dumps({"state": searcher_state.to_dict(),
                                                              "experiment_id": experiment_id}))
        self.save_method_state(path)

    def load(self, path: pathlib.Path) -> Tuple[SearcherState, int]:
        d = json.loads((path / "searcher_state.json").read_text())
        st = SearcherState()
        st.from_dict(d["state"])
        self.load_method_state(path)
        return st, int(d["experiment_id"])


def _tar_dir(model_dir: str) -> str:
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as tf:
        tf.add(model_dir, arcname=".", filter=lambda ti: None if "__pycache__" in ti.name else ti)
    return base64.b64encode(buf.getvalue()).decode()


class SearchRunner:
    def __init__(self, search_method: SearchMethod, session: Any = None) -> None:
        self.search_method = search_method
        self.state = SearcherState()
        self._session = session

    def _dispatch(self, ev: Dict[str, Any]) -> List[Operation]:
        st = self.state
        m = self.search_method
        if "initial_operations" in ev:
            return m.initial_operations(st)
        if "trial_created" in ev:
            rid = uuid.UUID(ev["trial_created"]["request_id"])
            st.trials_created.add(rid)
            st.trial_progress[rid] = 0.0
            return m.on_trial_created(st, rid)
        if "validation_completed" in ev:
            e = ev["validation_completed"]
            rid = uuid.UUID(e["request_id"])
            st.trial_progress[rid] = float(e["validate_after_length"])
            return m.on_validation_completed(st, rid, e["metric"], int(e["validate_after_length"]))
        if "trial_closed" in ev:
            rid = uuid.UUID(ev["trial_closed"]["request_id"])
            st.trials_closed.add(rid)
            return m.on_trial_closed(st, rid)
        if "trial_exited_early" in ev:
            e = ev["trial_exited_early"]
            rid = uuid.UUID(e["request_id"])
            st.failures.add(rid)
            st.trials_closed.add(rid)
            return m.on_trial_exited_early(st, rid, ExitedReason(e["exited_reason"]))
        if "experiment_inactive" in ev:
            st.experiment_completed = True
            return []
        logger.warning(f"unknown searcher event {ev}")
        return []

    def run_experiment(self, experiment_id: int, poll_timeout: float = 30.0) -> None:
        sess = self._session
        while not self.state.experiment_completed:
            events = sess.get(f"/api/v1/experiments/{experiment_id}/searcher_events",
                              params={"timeout_seconds": poll_timeout}, timeout=poll_timeout + 30)
            events = [e for e in (events or {}).get("events", []) if e["id"] > self.state.last_event_id]
            if not events:
                exp = sess.get(f"/api/v1/experiments/{experiment_id}")["experiment"]
                if exp["state"] in ("COMPLETED", "CANCELED", "ERROR", "DELETED"):
                    self.state.experiment_completed = True
                continue
            ops: List[Operation] = []
            for ev in events:
                ops += self._dispatch(ev)
                self.state.last_event_id = ev["id"]
            ops.append(Progress(self.search_method.progress(self.state)))
            sess.post(f"/api/v1/experiments/{experiment_id}/searcher_operations",
                      {"operations": [o.to_wire() for o in ops], "triggered_by_event": self.state.last_event_id})
            self.save_state(experiment_id)

    def save_state(self, experiment_id: int) -> None:
        pass


class LocalSearchRunner(SearchRunner):
    """Runs the search method in the calling process (reference LocalSearchRunner)."""

    def __init__(self, search_method: SearchMethod, searcher_dir: Optional[pathlib.Path] = None,
                 session: Any = None) -> None:
        if session is None:
            import os

            from determined_amd.common.api import Session

            session = Session(os.environ.get("DET_MASTER", "http://127.0.0.1:8080"))
        super().__init__(search_method, session)
        self.searcher_dir = pathlib.Path(searcher_dir or "./searcher_state")

    def run(self, exp_config: Dict[str, Any], model_dir: Optional[str] = None) -> int:
        state_file = self.searcher_dir / "searcher_state.json"
        if state_file.exists():
            self.state, exp_id = self.search_method.load(self.searcher_dir)
        else:
            cfg = dict(exp_config)
            cfg["searcher"] = dict(cfg.get("searcher", {}), name="custom")
            body = {"config": cfg, "model_def": _tar_dir(model_dir) if model_dir else None}
            exp_id = int(self._session.post("/api/v1/experiments", body)["experiment"]["id"])
        self._exp_id = exp_id
        self.run_experiment(exp_id)
        return exp_id

    def save_state(self, experiment_id: int) -> None:
        self.search_method.save(self.state, self.searcher_dir, experiment_id=experiment_id)


class RemoteSearchRunner(LocalSearchRunner):
    """Runs on-cluster inside a Core API task; state lives next to its checkpoints."""

    def __init__(self, search_method: SearchMethod, context: Any) -> None:
        from determined_amd.common.api import Session

        info = context.info
        session = Session(info.master_url, token=info.session_token) if info is not None else None
        super().__init__(search_method, pathlib.Path("/tmp") / "remote_searcher_state", session)
        self.context = context
