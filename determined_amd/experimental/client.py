"""Python SDK for the master (reference: ``harness/determined/experimental/client.py`` and
``common/experimental/{experiment,trial,checkpoint,model}.py``).

.. code-block:: python

    from determined_amd.experimental import client
    client.login("http://127.0.0.1:8080")
    exp = client.create_experiment("const.yaml", "examples/mnist_pytorch")
    exp.wait()
    ckpt = exp.top_checkpoint()
    path = ckpt.download()
    model = client.create_model("mnist")
    model.register_version(ckpt.uuid)

Objects are thin views over REST responses (``reload()`` refreshes them).  Checkpoint
download reads the experiment's ``checkpoint_storage`` directly (shared_fs / directory) like
the reference's ``DownloadMode.DIRECT``, falling back to nothing else since there is no
master-proxied download in this build.
"""

import base64
import contextvars
import enum
import io
import json
import logging
import os
import pathlib
import tarfile
import time
from typing import Any, Callable, Dict, Iterable, Iterator, List, Optional, Set, Union

import yaml

from determined_amd.common.api import NotFoundException, Session

_session: Optional[Session] = None
# set by ``Determined`` objects (experimental/determined.py) while one of their methods runs
_override: "contextvars.ContextVar[Optional[Session]]" = contextvars.ContextVar("damd_sdk_session", default=None)


def login(master: Optional[str] = None, user: Optional[str] = None, password: Optional[str] = None,
          token: Optional[str] = None) -> Session:
    """Set the module-level session (``DET_MASTER`` or ``http://127.0.0.1:8080`` by default)."""
    global _session
    url = master or os.environ.get("DET_MASTER") or "http://127.0.0.1:8080"
    s = Session(url, token=token)
    if user is not None and token is None:
        r = s.post("/api/v1/auth/login", {"username": user, "password": password or ""})
        s.token = (r or {}).get("token") or None
    _session = s
    return s


def logout() -> None:
    global _session
    _session = None


def _s() -> Session:
    bound = _override.get()
    if bound is not None:
        return bound
    if _session is None:
        login()
    assert _session is not None
    return _session


logger = logging.getLogger("determined_amd.client")

class ExperimentState(enum.Enum):
    ACTIVE = "ACTIVE"
    PAUSED = "PAUSED"
    STOPPING_COMPLETED = "STOPPING_COMPLETED"
    STOPPING_CANCELED = "STOPPING_CANCELED"
    STOPPING_ERROR = "STOPPING_ERROR"
    COMPLETED = "COMPLETED"
    CANCELED = "CANCELED"
    ERROR = "ERROR"
    DELETED = "DELETED"


TERMINAL = {ExperimentState.COMPLETED, ExperimentState.CANCELED, ExperimentState.ERROR, ExperimentState.DELETED}


class TrialState(enum.Enum):
    ACTIVE = "ACTIVE"
    PAUSED = "PAUSED"
    COMPLETED = "COMPLETED"
    CANCELED = "CANCELED"
    ERROR = "ERROR"


class CheckpointState(enum.Enum):
    ACTIVE = "ACTIVE"
    COMPLETED = "COMPLETED"
    DELETED = "DELETED"
    PARTIALLY_DELETED = "PARTIALLY_DELETED"
    ERROR = "ERROR"


class DownloadMode(enum.Enum):
    AUTO = "auto"
    DIRECT = "direct"
    MASTER = "master"


def _tar_dir(path: str) -> bytes:
    from determined_amd.cli import tar_model_dir

    return tar_model_dir(path)


# ---------------------------------------------------------------------------------------------
# checkpoints
# ---------------------------------------------------------------------------------------------
class Checkpoint:
    def __init__(self, session: Session, uuid: str, data: Optional[Dict[str, Any]] = None) -> None:
        self._session = session
        self.uuid = uuid
        self._data = data or {}
        if not data:
            self.reload()

    def reload(self) -> None:
        self._data = self._session.get(f"/api/v1/checkpoints/{self.uuid}")["checkpoint"]

    @property
    def metadata(self) -> Dict[str, Any]:
        return dict(self._data.get("metadata") or {})

    @property
    def state(self) -> CheckpointState:
        return CheckpointState(self._data.get("state") or "COMPLETED")

    @property
    def trial_id(self) -> Optional[int]:
        return self._data.get("trial_id")

    @property
    def steps_completed(self) -> Optional[int]:
        return self._data.get("steps_completed")

    @property
    def resources(self) -> Dict[str, int]:
        return dict(self._data.get("resources") or {})

    @property
    def searcher_metric(self) -> Optional[float]:
        return self._data.get("searcher_metric")

    def _storage(self) -> Any:
        from determined_amd import storage

        cfg = self._data.get("checkpoint_storage")
        if cfg is None:
            self.reload()
            cfg = self._data.get("checkpoint_storage")
        if cfg is None:
            raise RuntimeError(f"checkpoint {self.uuid} has no experiment storage configuration")
        return storage.build(cfg)

    def download(self, path: Optional[str] = None, mode: DownloadMode = DownloadMode.AUTO) -> str:
        """Fetch the checkpoint into ``path`` (default ``checkpoints/<uuid>``).  DIRECT reads the checkpoint
        storage from this machine; MASTER streams a tar.gz through the master (for clients without
        access to the storage); AUTO tries DIRECT and falls back to MASTER (reference
        ``checkpoint/_checkpoint.py`` download / ``_download_auto``)."""
        path = path or os.path.join("checkpoints", self.uuid)
        if not os.path.exists(os.path.join(path, "metadata.json")):
            if mode == DownloadMode.DIRECT:
                self._download_direct(path)
            elif mode == DownloadMode.MASTER:
                self._download_via_master(path)
            elif mode == DownloadMode.AUTO:
                try:
                    self._download_direct(path)
                except (OSError, RuntimeError) as e:
                    if (self._data.get("checkpoint_storage") or {}).get("type") == "azure":
                        raise
                    logger.info(f"direct download of checkpoint {self.uuid} failed ({e}); proxying through the master")
                    try:
                        self._download_via_master(path)
                    except Exception as e2:
                        raise RuntimeError(f"checkpoint {self.uuid}: direct download and download through the "
                                           f"master both failed ({e}; {e2})") from e2
            else:
                raise ValueError(f"unknown download mode {mode}")
        md = os.path.join(path, "metadata.json")
        if not os.path.exists(md):
            self.write_metadata_file(md)
        return path

    def _download_direct(self, path: str) -> None:
        sm = self._storage()
        base = getattr(sm, "_base_path", None)
        if base is not None and not os.path.isdir(os.path.join(str(base), self.uuid)):
            raise FileNotFoundError(f"checkpoint {self.uuid} not found under {base} on this machine")
        os.makedirs(path, exist_ok=True)
        sm.download(src=self.uuid, dst=path)

    def _download_via_master(self, path: str) -> None:
        import io
        import tarfile

        url = f"{self._session.master_url}/api/v1/checkpoints/{self.uuid}/download"
        r = self._session._http.get(url, headers={**self._session._headers(), "Accept": "application/gzip"},
                                    timeout=self._session.timeout)
        if r.status_code >= 400:
            raise RuntimeError(f"master could not serve checkpoint {self.uuid}: {r.status_code} {r.text}")
        os.makedirs(path, exist_ok=True)
        with tarfile.open(fileobj=io.BytesIO(r.content), mode="r:gz") as tf:
            tf.extractall(path, filter="data")

    def write_metadata_file(self, path: str) -> None:
        with open(path, "w") as f:
            json.dump(self.metadata, f, indent=2, sort_keys=True)

    def add_metadata(self, metadata: Dict[str, Any]) -> None:
        md = self.metadata
        md.update(metadata)
        self._session.patch(f"/api/v1/checkpoints/{self.uuid}", {"metadata": md})
        self._data["metadata"] = md

    def remove_metadata(self, keys: List[str]) -> None:
        md = {k: v for k, v in self.metadata.items() if k not in keys}
        self._session.patch(f"/api/v1/checkpoints/{self.uuid}", {"metadata": md})
        self._data["metadata"] = md

    def delete(self) -> None:
        self._session.delete(f"/api/v1/checkpoints/{self.uuid}")

    def get_metrics(self, group: Optional[str] = None) -> Iterator["TrialMetrics"]:
        """Metrics of the tasks that reported using this checkpoint
        (``core_context.experimental.report_task_using_checkpoint``; reference
        ``checkpoint/_checkpoint.py:get_metrics``); every group when ``group`` is None / ""."""
        params = {"group": group} if group else {}
        for r in self._session.get(f"/api/v1/checkpoints/{self.uuid}/metrics", params=params)["metrics"]:
            yield TrialMetrics._from_row(r["trial_id"], r)

    def __repr__(self) -> str:
        return f"Checkpoint(uuid={self.uuid})"


# ---------------------------------------------------------------------------------------------
# trials
# ---------------------------------------------------------------------------------------------
class Trial:
    def __init__(self, session: Session, trial_id: int, data: Optional[Dict[str, Any]] = None) -> None:
        self._session = session
        self.id = trial_id
        self._data = data or {}
        if not data:
            self.reload()

    def reload(self) -> None:
        self._data = self._session.get(f"/api/v1/trials/{self.id}")["trial"]

    @property
    def experiment_id(self) -> int:
        return int(self._data["experiment_id"])

    @property
    def hparams(self) -> Dict[str, Any]:
        return dict(self._data.get("hparams") or {})

    @property
    def state(self) -> TrialState:
        return TrialState(self._data["state"])

    @property
    def summary_metrics(self) -> Dict[str, Any]:
        return {"latest_validation": self._data.get("latest_validation"),
                "latest_training": self._data.get("latest_training")}

    def iter_logs(self, follow: bool = False, head: Optional[int] = None, tail: Optional[int] = None,
                  search_text: Optional[str] = None) -> Iterator[str]:
        after = 0
        emitted: List[str] = []
        while True:
            rows = self._session.get(f"/api/v1/tasks/trial-{self.id}/logs", params={"after": after})["logs"]
            for r in rows:
                after = max(after, int(r["id"]))
                if search_text and search_text not in r["log"]:
                    continue
                emitted.append(r["log"])
                if tail is None:
                    yield r["log"]
                    if head is not None and len(emitted) >= head:
                        return
            if not follow:
                break
            self.reload()
            if self._data["state"] in ("COMPLETED", "CANCELED", "ERROR") and not rows:
                break
            time.sleep(0.5)
        if tail is not None:
            yield from emitted[-tail:]

    def logs(self, *args: Any, **kwargs: Any) -> Iterable[str]:
        return self.iter_logs(*args, **kwargs)

    def kill(self) -> None:
        self._session.post(f"/api/v1/trials/{self.id}/kill", {})

    def list_checkpoints(self) -> List[Checkpoint]:
        rows = self._session.get(f"/api/v1/trials/{self.id}/checkpoints")["checkpoints"]
        return [Checkpoint(self._session, r["uuid"], r) for r in rows]

    def top_checkpoint(self, sort_by: Optional[str] = None, smaller_is_better: Optional[bool] = None) -> Checkpoint:
        cks = self.list_checkpoints()
        if not cks:
            raise RuntimeError(f"trial {self.id} has no checkpoints")
        return _best(cks, self._session, self.experiment_id, sort_by, smaller_is_better)[0]

    def select_checkpoint(self, latest: bool = False, best: bool = False, uuid: Optional[str] = None,
                          sort_by: Optional[str] = None, smaller_is_better: Optional[bool] = None) -> Checkpoint:
        if sum([latest, best, uuid is not None]) != 1:
            raise ValueError("pass exactly one of latest / best / uuid")
        if uuid is not None:
            return Checkpoint(self._session, uuid)
        if latest:
            cks = self.list_checkpoints()
            return max(cks, key=lambda c: c.steps_completed or 0)
        return self.top_checkpoint(sort_by, smaller_is_better)

    def iter_metrics(self, group: str) -> Iterator["TrialMetrics"]:
        """``TrialMetrics`` reports of one group (``TrainingMetrics`` / ``ValidationMetrics``)."""
        rows = self._session.get(f"/api/v1/trials/{self.id}/metrics", params={"group": group})["metrics"]
        for r in rows:
            yield TrialMetrics._from_row(self.id, r)

    def stream_training_metrics(self) -> Iterable[Dict[str, Any]]:
        return self.iter_metrics("training")

    def stream_validation_metrics(self) -> Iterable[Dict[str, Any]]:
        return self.iter_metrics("validation")

    def __repr__(self) -> str:
        return f"Trial(id={self.id})"


def _best(cks: List[Checkpoint], session: Session, exp_id: int, sort_by: Optional[str],
          smaller_is_better: Optional[bool]) -> List[Checkpoint]:
    cfg = session.get(f"/api/v1/experiments/{exp_id}")["config"]
    metric = sort_by or cfg["searcher"]["metric"]
    sib = cfg["searcher"].get("smaller_is_better", True) if smaller_is_better is None else smaller_is_better

    def val(c: Checkpoint) -> float:
        v = c.searcher_metric if sort_by is None else None
        if v is None:
            for mrow in Trial(session, c.trial_id).iter_metrics("validation") if c.trial_id else []:
                if mrow["steps_completed"] == c.steps_completed and metric in (mrow["metrics"] or {}):
                    v = mrow["metrics"][metric]
        if v is None:
            return float("inf") if sib else float("-inf")
        return float(v)

    return sorted(cks, key=val, reverse=not sib)


# ---------------------------------------------------------------------------------------------
# experiments
# ---------------------------------------------------------------------------------------------
class Experiment:
    def __init__(self, session: Session, experiment_id: int, data: Optional[Dict[str, Any]] = None) -> None:
        self._session = session
        self._id = experiment_id
        self._data = data or {}
        self._config: Optional[Dict[str, Any]] = None
        if not data:
            self.reload()

    @property
    def id(self) -> int:
        return self._id

    def reload(self) -> None:
        r = self._session.get(f"/api/v1/experiments/{self._id}")
        self._data, self._config = r["experiment"], r.get("config")

    @property
    def state(self) -> ExperimentState:
        return ExperimentState(self._data["state"])

    @property
    def name(self) -> str:
        return self._data.get("name") or ""

    @property
    def config(self) -> Dict[str, Any]:
        if self._config is None:
            self.reload()
        return dict(self._config or {})

    @property
    def progress(self) -> float:
        return float(self._data.get("progress") or 0.0)

    @property
    def labels(self) -> Set[str]:
        return set(self._data.get("labels") or [])

    def _patch(self, **cols: Any) -> None:
        self._session.patch(f"/api/v1/experiments/{self._id}", cols)
        self._data.update(cols)

    def set_name(self, name: str) -> None:
        self._patch(name=name)

    def set_description(self, description: str) -> None:
        self._patch(description=description)

    def set_notes(self, notes: str) -> None:
        self._patch(notes=notes)

    def add_label(self, label: str) -> None:
        self.set_labels(self.labels | {label})

    def remove_label(self, label: str) -> None:
        self.set_labels(self.labels - {label})

    def set_labels(self, labels: Set[str]) -> None:
        self._patch(labels=sorted(labels))

    def _action(self, verb: str) -> None:
        self._session.post(f"/api/v1/experiments/{self._id}/{verb}", {})

    def activate(self) -> None:
        self._action("activate")

    def pause(self) -> None:
        self._action("pause")

    def kill(self) -> None:
        self._action("kill")

    def cancel(self) -> None:
        self._action("cancel")

    def archive(self) -> None:
        self._action("archive")

    def unarchive(self) -> None:
        self._action("unarchive")

    def delete(self) -> None:
        self._session.delete(f"/api/v1/experiments/{self._id}")

    def download_code(self, output_dir: Optional[str] = None) -> str:
        b64 = self._session.get(f"/api/v1/experiments/{self._id}/model_def")["b64_tgz"]
        out = output_dir or f"exp-{self._id}-code"
        os.makedirs(out, exist_ok=True)
        if b64:
            with tarfile.open(fileobj=io.BytesIO(base64.b64decode(b64)), mode="r:gz") as tf:
                tf.extractall(out, filter="data") if hasattr(tarfile, "data_filter") else tf.extractall(out)
        return out

    def list_trials(self) -> List[Trial]:
        rows = self._session.get(f"/api/v1/experiments/{self._id}/trials")["trials"]
        return [Trial(self._session, r["id"], r) for r in rows]

    get_trials = list_trials

    def iter_trials(self) -> Iterator[Trial]:
        yield from self.list_trials()

    def await_first_trial(self, interval: float = 0.1, timeout: float = 600.0) -> Trial:
        t0 = time.time()
        while time.time() - t0 < timeout:
            ts = self.list_trials()
            if ts:
                return ts[0]
            time.sleep(interval)
        raise TimeoutError(f"experiment {self._id} created no trial within {timeout}s")

    def wait(self, interval: float = 5.0, timeout: Optional[float] = None) -> ExperimentState:
        t0 = time.time()
        while True:
            self.reload()
            if self.state in TERMINAL:
                return self.state
            if timeout is not None and time.time() - t0 > timeout:
                raise TimeoutError(f"experiment {self._id} still {self.state.value}")
            time.sleep(interval)

    def list_checkpoints(self, sort_by: Optional[str] = None, smaller_is_better: Optional[bool] = None,
                         max_results: Optional[int] = None) -> List[Checkpoint]:
        rows = self._session.get(f"/api/v1/experiments/{self._id}/checkpoints")["checkpoints"]
        cks = [Checkpoint(self._session, r["uuid"], r) for r in rows if r.get("state", "COMPLETED") != "DELETED"]
        if sort_by is not None or smaller_is_better is not None:
            cks = _best(cks, self._session, self._id, sort_by, smaller_is_better)
        return cks[:max_results] if max_results else cks

    def top_checkpoint(self, sort_by: Optional[str] = None, smaller_is_better: Optional[bool] = None) -> Checkpoint:
        cks = self.top_n_checkpoints(1, sort_by, smaller_is_better)
        if not cks:
            raise RuntimeError(f"experiment {self._id} has no checkpoints")
        return cks[0]

    def top_n_checkpoints(self, limit: int, sort_by: Optional[str] = None,
                          smaller_is_better: Optional[bool] = None) -> List[Checkpoint]:
        cks = self.list_checkpoints()
        return _best(cks, self._session, self._id, sort_by, smaller_is_better)[:limit]

    def __repr__(self) -> str:
        return f"Experiment(id={self._id})"


def create_experiment(config: Union[str, pathlib.Path, Dict[str, Any]], model_dir: Optional[str] = None,
                      includes: Optional[Iterable[Union[str, pathlib.Path]]] = None, parent_id: Optional[int] = None,
                      activate: bool = True) -> Experiment:
    if isinstance(config, (str, pathlib.Path)):
        with open(config) as f:
            config = yaml.safe_load(f)
    body: Dict[str, Any] = {"config": config, "activate": activate, "parent_id": parent_id}
    if model_dir is not None:
        body["model_def"] = base64.b64encode(_tar_dir(model_dir)).decode()
    r = _s().post("/api/v1/experiments", body)
    return Experiment(_s(), r["experiment"]["id"], r["experiment"])


def get_experiment(experiment_id: int) -> Experiment:
    return Experiment(_s(), experiment_id)


def list_experiments(archived: Optional[bool] = None, name: Optional[str] = None) -> List[Experiment]:
    params = {} if archived is None else {"archived": str(archived).lower()}
    rows = _s().get("/api/v1/experiments", params=params)["experiments"]
    return [Experiment(_s(), r["id"], r) for r in rows if name is None or r.get("name") == name]


def get_trial(trial_id: int) -> Trial:
    return Trial(_s(), trial_id)


def get_checkpoint(uuid: str) -> Checkpoint:
    return Checkpoint(_s(), uuid)


# ---------------------------------------------------------------------------------------------
# model registry
# ---------------------------------------------------------------------------------------------
class ModelVersion:
    def __init__(self, session: Session, model_name: str, data: Dict[str, Any]) -> None:
        self._session = session
        self.model_name = model_name
        self._data = data

    @property
    def model_version(self) -> int:
        return int(self._data["version"])

    @property
    def name(self) -> str:
        return self._data.get("name") or ""

    @property
    def notes(self) -> str:
        return self._data.get("comment") or ""

    @property
    def checkpoint(self) -> Checkpoint:
        return Checkpoint(self._session, self._data["checkpoint_uuid"])

    def _path(self) -> str:
        return f"/api/v1/models/{self.model_name}/versions/{self.model_version}"

    def set_name(self, name: str) -> None:
        self._session.patch(self._path(), {"name": name})
        self._data["name"] = name

    def set_notes(self, notes: str) -> None:
        self._session.patch(self._path(), {"notes": notes})
        self._data["comment"] = notes

    def delete(self) -> None:
        self._session.delete(self._path())

    def get_metrics(self, group: Optional[str] = None) -> Iterator["TrialMetrics"]:
        """Metrics of the tasks that reported using this model version
        (``core_context.experimental.report_task_using_model_version``)."""
        params = {"group": group} if group else {}
        for r in self._session.get(f"{self._path()}/metrics", params=params)["metrics"]:
            yield TrialMetrics._from_row(r["trial_id"], r)

    @property
    def model_id(self) -> Optional[int]:
        mid = self._data.get("model_id")
        return int(mid) if mid is not None else None

    def __repr__(self) -> str:
        return f"ModelVersion({self.model_name}, v{self.model_version})"


class Model:
    def __init__(self, session: Session, data: Dict[str, Any]) -> None:
        self._session = session
        self._data = data

    @property
    def name(self) -> str:
        return self._data["name"]

    @property
    def model_id(self) -> int:
        return int(self._data["id"])

    @property
    def description(self) -> str:
        return self._data.get("description") or ""

    @property
    def metadata(self) -> Dict[str, Any]:
        return dict(self._data.get("metadata") or {})

    @property
    def labels(self) -> List[str]:
        return list(self._data.get("labels") or [])

    def reload(self) -> None:
        self._data = self._session.get(f"/api/v1/models/{self.name}")["model"]

    def list_versions(self) -> List[ModelVersion]:
        rows = self._session.get(f"/api/v1/models/{self.name}/versions")["model_versions"]
        return [ModelVersion(self._session, self.name, r) for r in sorted(rows, key=lambda r: -r["version"])]

    get_versions = list_versions

    def get_version(self, version: int = -1) -> Optional[ModelVersion]:
        vs = self.list_versions()
        if not vs:
            return None
        if version == -1:
            return vs[0]
        return next((v for v in vs if v.model_version == version), None)

    def register_version(self, checkpoint_uuid: str) -> ModelVersion:
        r = self._session.post(f"/api/v1/models/{self.name}/versions", {"checkpoint_uuid": checkpoint_uuid})
        return ModelVersion(self._session, self.name, r["model_version"])

    def _patch(self, **cols: Any) -> None:
        self._session.patch(f"/api/v1/models/{self.name}", cols)
        self._data.update(cols)

    def set_description(self, description: str) -> None:
        self._patch(description=description)

    def add_metadata(self, metadata: Dict[str, Any]) -> None:
        md = self.metadata
        md.update(metadata)
        self._patch(metadata=md)

    def remove_metadata(self, keys: List[str]) -> None:
        self._patch(metadata={k: v for k, v in self.metadata.items() if k not in keys})

    def set_labels(self, labels: List[str]) -> None:
        self._patch(labels=list(labels))

    def archive(self) -> None:
        self._patch(archived=1)

    def unarchive(self) -> None:
        self._patch(archived=0)

    def delete(self) -> None:
        self._session.delete(f"/api/v1/models/{self.name}")

    def __repr__(self) -> str:
        return f"Model(name={self.name})"


def create_model(name: str, description: str = "", metadata: Optional[Dict[str, Any]] = None,
                 labels: Optional[List[str]] = None) -> Model:
    r = _s().post("/api/v1/models", {"name": name, "description": description, "metadata": metadata or {},
                                     "labels": labels or []})
    return Model(_s(), r["model"])


def get_model(identifier: Union[str, int]) -> Model:
    if isinstance(identifier, int):
        for m in list_models():
            if m.model_id == identifier:
                return m
        raise NotFoundException(404, f"model {identifier} not found")
    return Model(_s(), _s().get(f"/api/v1/models/{identifier}")["model"])


def list_models(name: Optional[str] = None, labels: Optional[List[str]] = None) -> List[Model]:
    rows = _s().get("/api/v1/models")["models"]
    out = [Model(_s(), r) for r in rows]
    if name is not None:
        out = [m for m in out if m.name == name]
    if labels:
        out = [m for m in out if set(labels) <= set(m.labels)]
    return out


get_models = list_models


def get_model_labels() -> List[str]:
    return sorted({lab for m in list_models() for lab in m.labels})


def stream_trials_training_metrics(trial_ids: List[int]) -> Iterable[Dict[str, Any]]:
    for tid in trial_ids:
        yield from Trial(_s(), tid).iter_metrics("training")


def stream_trials_validation_metrics(trial_ids: List[int]) -> Iterable[Dict[str, Any]]:
    for tid in trial_ids:
        yield from Trial(_s(), tid).iter_metrics("validation")


def iter_trials_metrics(trial_ids: List[int], group: str) -> Iterable[Dict[str, Any]]:
    for tid in trial_ids:
        yield from Trial(_s(), tid).iter_metrics(group)


# ---------------------------------------------------------------------------------------------
# users, workspaces, projects (reference: common/experimental/{user,workspace,project}.py and the
# user / workspace functions of experimental/client.py)
# ---------------------------------------------------------------------------------------------
class User:
    def __init__(self, session: Session, data: Dict[str, Any]) -> None:
        self._session = session
        self._data = data

    @property
    def user_id(self) -> int:
        return int(self._data["id"])

    @property
    def username(self) -> str:
        return self._data["username"]

    @property
    def display_name(self) -> str:
        return self._data.get("display_name") or ""

    @property
    def admin(self) -> bool:
        return bool(self._data.get("admin"))

    @property
    def active(self) -> bool:
        return bool(self._data.get("active"))

    def reload(self) -> None:
        self._data = self._session.get(f"/api/v1/users/{self.user_id}")["user"]

    def _patch(self, **cols: Any) -> None:
        self._data = self._session.patch(f"/api/v1/users/{self.user_id}", cols)["user"]

    def rename(self, new_username: str) -> None:
        self._patch(username=new_username)

    def activate(self) -> None:
        self._patch(active=True)

    def deactivate(self) -> None:
        self._patch(active=False)

    def change_display_name(self, display_name: str) -> None:
        self._patch(display_name=display_name)

    def change_password(self, new_password: str) -> None:
        self._data = self._session.post(f"/api/v1/users/{self.user_id}/password", {"password": new_password})["user"]

    def __repr__(self) -> str:
        return f"User(id={self.user_id}, username={self.username})"


def create_user(username: str, admin: bool = False, password: Optional[str] = None,
                display_name: Optional[str] = None) -> User:
    r = _s().post("/api/v1/users", {"user": {"username": username, "admin": admin, "active": True,
                                             "display_name": display_name or ""}, "password": password or ""})
    return User(_s(), r["user"])


def get_user_by_id(user_id: int) -> User:
    return User(_s(), _s().get(f"/api/v1/users/{int(user_id)}")["user"])


def get_user_by_name(user_name: str) -> User:
    return User(_s(), _s().get(f"/api/v1/users/{user_name}")["user"])


def whoami() -> User:
    return User(_s(), _s().get("/api/v1/me")["user"])


def get_session_username() -> str:
    return whoami().username


def list_users(active: Optional[bool] = None) -> List[User]:
    rows = _s().get("/api/v1/users")["users"]
    return [User(_s(), r) for r in rows if active is None or bool(r.get("active")) == active]


class Project:
    def __init__(self, session: Session, data: Dict[str, Any]) -> None:
        self._session = session
        self._data = data

    @property
    def id(self) -> int:
        return int(self._data["id"])

    @property
    def name(self) -> str:
        return self._data["name"]

    @property
    def description(self) -> str:
        return self._data.get("description") or ""

    @property
    def workspace_id(self) -> int:
        return int(self._data["workspace_id"])

    @property
    def archived(self) -> bool:
        return bool(self._data.get("archived"))

    def reload(self) -> None:
        self._data = self._session.get(f"/api/v1/projects/{self.id}")["project"]

    def list_experiments(self) -> List["Experiment"]:
        rows = self._session.get(f"/api/v1/projects/{self.id}/experiments")["experiments"]
        return [Experiment(self._session, int(r["id"])) for r in rows]

    def set_name(self, name: str) -> None:
        self._data = self._session.patch(f"/api/v1/projects/{self.id}", {"name": name})["project"]

    def set_description(self, description: str) -> None:
        self._data = self._session.patch(f"/api/v1/projects/{self.id}", {"description": description})["project"]

    def archive(self) -> None:
        self._data = self._session.post(f"/api/v1/projects/{self.id}/archive", {})["project"]

    def unarchive(self) -> None:
        self._data = self._session.post(f"/api/v1/projects/{self.id}/unarchive", {})["project"]

    def __repr__(self) -> str:
        return f"Project(id={self.id}, name={self.name})"


class Workspace:
    def __init__(self, session: Session, data: Dict[str, Any]) -> None:
        self._session = session
        self._data = data

    @property
    def id(self) -> int:
        return int(self._data["id"])

    @property
    def name(self) -> str:
        return self._data["name"]

    @property
    def archived(self) -> bool:
        return bool(self._data.get("archived"))

    def reload(self) -> None:
        self._data = self._session.get(f"/api/v1/workspaces/{self.id}")["workspace"]

    def list_projects(self) -> List[Project]:
        rows = self._session.get(f"/api/v1/workspaces/{self.id}/projects")["projects"]
        return [Project(self._session, r) for r in rows]

    def get_project(self, project_name: str) -> Project:
        for p in self.list_projects():
            if p.name == project_name:
                return p
        raise NotFoundException(404, f"project {project_name!r} not found in workspace {self.name!r}")

    def create_project(self, name: str, description: Optional[str] = None) -> Project:
        r = self._session.post(f"/api/v1/workspaces/{self.id}/projects",
                               {"name": name, "description": description or ""})
        return Project(self._session, r["project"])

    def delete_project(self, name: str) -> None:
        self._session.delete(f"/api/v1/projects/{self.get_project(name).id}")

    def list_pools(self) -> List["ResourcePool"]:
        """Resource pools usable from this workspace (unbound pools + pools bound to it)."""
        rows = self._session.get(f"/api/v1/workspaces/{self.id}/available-resource-pools").get("resource_pools") or []
        return [ResourcePool(self._session, r["name"] if isinstance(r, dict) else str(r)) for r in rows]

    def __repr__(self) -> str:
        return f"Workspace(id={self.id}, name={self.name})"


def get_workspace(name: str) -> Workspace:
    return Workspace(_s(), _s().get(f"/api/v1/workspaces/{name}")["workspace"])


def list_workspaces() -> List[Workspace]:
    return [Workspace(_s(), r) for r in _s().get("/api/v1/workspaces")["workspaces"]]


def create_workspace(name: str) -> Workspace:
    return Workspace(_s(), _s().post("/api/v1/workspaces", {"name": name})["workspace"])


def delete_workspace(name: str) -> None:
    _s().delete(f"/api/v1/workspaces/{name}")


def get_model_by_id(model_id: int) -> Model:
    return get_model(int(model_id))


def stream_trials_metrics(trial_ids: List[int], group: str) -> Iterable[Dict[str, Any]]:
    return iter_trials_metrics(trial_ids, group)


def list_resource_pools() -> List["ResourcePool"]:
    return _list_resource_pools(_s())


def get_resource_pool(name: str) -> "ResourcePool":
    return ResourcePool(_s(), name)


from determined_amd.experimental.determined import (  # noqa: E402  (cyclic: determined.py imports this lazily)
    Determined,
    ResourcePool,
    TrainingMetrics,
    TrialMetrics,
    ValidationMetrics,
    list_resource_pools as _list_resource_pools,
    test_one_batch,
)
