"""Object-style SDK entry point and the remaining SDK objects (reference:
``harness/determined/common/experimental/determined.py`` (``Determined``),
``resource_pool.py`` (``ResourcePool``), ``metrics.py`` (``TrialMetrics`` /
``TrainingMetrics`` / ``ValidationMetrics``) and ``experimental/_native.py``
(``test_one_batch``)).

``Determined(master, user, password)`` owns its own :class:`Session`; every method runs the
module-level function of :mod:`determined_amd.experimental.client` with that session bound, so
objects it returns talk to the same master (several masters can be used side by side, unlike the
``client`` module's single login).
"""

import contextlib
import dataclasses
import datetime
import logging
import os
from typing import Any, Callable, Dict, Iterable, Iterator, List, Optional, Type, Union

from determined_amd.common.api import Session

logger = logging.getLogger("determined_amd")


# ----------------------------------------------------------------------------------- metrics
@dataclasses.dataclass
class TrialMetrics:
    """One metrics report of a trial (reference ``common/experimental/metrics.py:TrialMetrics``).
    Item access (``m["metrics"]``) keeps the earlier dict view working."""

    trial_id: int
    trial_run_id: Optional[int]
    steps_completed: int
    end_time: Optional[datetime.datetime]
    metrics: Dict[str, Any]
    group: str
    batch_metrics: Optional[List[Dict[str, Any]]] = None

    def __getitem__(self, key: str) -> Any:
        if key == "time":
            return self.end_time
        return getattr(self, key)

    def get(self, key: str, default: Any = None) -> Any:
        try:
            return self[key]
        except AttributeError:
            return default

    @classmethod
    def _from_row(cls, trial_id: int, row: Dict[str, Any]) -> "TrialMetrics":
        group = row.get("group_name") or row.get("group") or ""
        sub = {"training": TrainingMetrics, "validation": ValidationMetrics}.get(group, TrialMetrics)
        ts = row.get("ts")
        end = None
        if isinstance(ts, (int, float)):
            end = datetime.datetime.fromtimestamp(float(ts), tz=datetime.timezone.utc)
        elif isinstance(ts, str) and ts:
            try:
                end = datetime.datetime.fromisoformat(ts.replace("Z", "+00:00"))
            except ValueError:
                end = None
        return sub(trial_id=int(trial_id), trial_run_id=row.get("trial_run_id"),
                   steps_completed=int(row.get("steps_completed") or 0), end_time=end,
                   metrics=dict(row.get("metrics") or {}), group=group,
                   batch_metrics=row.get("batch_metrics"))


@dataclasses.dataclass
class TrainingMetrics(TrialMetrics):
    """A ``training`` group report."""


@dataclasses.dataclass
class ValidationMetrics(TrialMetrics):
    """A ``validation`` group report."""


# ------------------------------------------------------------------------------ resource pools
class ResourcePool:
    """A resource pool and its workspace bindings (reference ``resource_pool.py``).  A pool with
    bindings is usable only from the workspaces bound to it."""

    def __init__(self, session: Session, name: str = "") -> None:
        self.name = name
        self._session = session

    def _path(self) -> str:
        return f"/api/v1/resource-pools/{self.name}/workspace-bindings"

    def add_bindings(self, workspace_names: List[str]) -> None:
        self._session.post(self._path(), {"workspace_names": list(workspace_names)})

    def remove_bindings(self, workspace_names: List[str]) -> None:
        self._session.request("DELETE", self._path(), {"workspace_names": list(workspace_names)})

    def replace_bindings(self, workspace_names: List[str]) -> None:
        self._session.request("PUT", self._path(), {"workspace_names": list(workspace_names)})

    def list_workspaces(self) -> List[Optional[str]]:
        return list(self._session.get(self._path()).get("workspaces") or [])

    def describe(self) -> Dict[str, Any]:
        """The pool's row of ``GET /api/v1/resource-pools`` (slots, scheduler, queue lengths)."""
        for r in self._session.get("/api/v1/resource-pools").get("resource_pools") or []:
            if r.get("name") == self.name:
                return r
        from determined_amd.common.api import NotFoundException

        raise NotFoundException(404, f"resource pool {self.name!r} not found")

    def __repr__(self) -> str:
        return f"ResourcePool(name={self.name})"


def list_resource_pools(session: Session) -> List[ResourcePool]:
    return [ResourcePool(session, r["name"]) for r in session.get("/api/v1/resource-pools").get("resource_pools") or []]


# --------------------------------------------------------------------------------- Determined
class Determined:
    """Client object bound to one master (reference ``Determined``): the same methods as the
    ``client`` module's functions, each using this object's session."""

    def __init__(self, master: Optional[str] = None, user: Optional[str] = None,
                 password: Optional[str] = None, token: Optional[str] = None) -> None:
        url = master or os.environ.get("DET_MASTER") or "http://127.0.0.1:8080"
        s = Session(url, token=token)
        if user is not None and token is None:
            r = s.post("/api/v1/auth/login", {"username": user, "password": password or ""})
            s.token = (r or {}).get("token") or None
        self._session = s

    @classmethod
    def _from_session(cls, session: Session) -> "Determined":
        d = cls.__new__(cls)
        d._session = session
        return d

    @contextlib.contextmanager
    def _bound(self) -> Iterator[None]:
        from determined_amd.experimental import client

        tok = client._override.set(self._session)
        try:
            yield
        finally:
            client._override.reset(tok)

    def _call(self, name: str) -> Callable[..., Any]:
        from determined_amd.experimental import client

        fn = getattr(client, name)

        def run(*args: Any, **kwargs: Any) -> Any:
            with self._bound():
                out = fn(*args, **kwargs)
                # generators must run with the session bound too
                if hasattr(out, "__next__"):
                    out = list(out)
                return out

        return run

    # users
    def create_user(self, username: str, admin: bool = False, password: Optional[str] = None) -> Any:
        return self._call("create_user")(username, admin, password)

    def get_user_by_id(self, user_id: int) -> Any:
        return self._call("get_user_by_id")(user_id)

    def get_user_by_name(self, user_name: str) -> Any:
        return self._call("get_user_by_name")(user_name)

    def whoami(self) -> Any:
        return self._call("whoami")()

    def get_session_username(self) -> str:
        return self._call("get_session_username")()

    def logout(self) -> None:
        try:
            self._session.post("/api/v1/auth/logout", {})
        finally:
            self._session.token = None

    def list_users(self, active: Optional[bool] = None) -> List[Any]:
        return self._call("list_users")(active)

    # experiments / trials / checkpoints
    def create_experiment(self, config: Union[str, Dict[str, Any]], model_dir: Optional[str] = None,
                          includes: Optional[Iterable[str]] = None, parent_id: Optional[int] = None,
                          activate: bool = True) -> Any:
        return self._call("create_experiment")(config, model_dir, includes, parent_id, activate)

    def get_experiment(self, experiment_id: int) -> Any:
        return self._call("get_experiment")(experiment_id)

    def list_experiments(self, archived: Optional[bool] = None, name: Optional[str] = None) -> List[Any]:
        return self._call("list_experiments")(archived, name)

    def get_trial(self, trial_id: int) -> Any:
        return self._call("get_trial")(trial_id)

    def get_checkpoint(self, uuid: str) -> Any:
        return self._call("get_checkpoint")(uuid)

    # workspaces
    def get_workspace(self, name: str) -> Any:
        return self._call("get_workspace")(name)

    def list_workspaces(self) -> List[Any]:
        return self._call("list_workspaces")()

    def create_workspace(self, name: str) -> Any:
        return self._call("create_workspace")(name)

    def delete_workspace(self, name: str) -> None:
        self._call("delete_workspace")(name)

    # model registry
    def create_model(self, name: str, description: str = "", metadata: Optional[Dict[str, Any]] = None,
                     labels: Optional[List[str]] = None) -> Any:
        return self._call("create_model")(name, description, metadata, labels)

    def get_model(self, identifier: Union[str, int]) -> Any:
        return self._call("get_model")(identifier)

    def get_model_by_id(self, model_id: int) -> Any:
        return self._call("get_model_by_id")(model_id)

    def list_models(self, name: Optional[str] = None, labels: Optional[List[str]] = None) -> List[Any]:
        return self._call("list_models")(name, labels)

    get_models = list_models

    def get_model_labels(self) -> List[str]:
        return self._call("get_model_labels")()

    # resource pools
    def get_resource_pool(self, name: str) -> ResourcePool:
        return ResourcePool(self._session, name)

    def list_resource_pools(self) -> List[ResourcePool]:
        return list_resource_pools(self._session)

    # metrics
    def iter_trials_metrics(self, trial_ids: List[int], group: str) -> List[TrialMetrics]:
        return self._call("iter_trials_metrics")(trial_ids, group)

    def stream_trials_metrics(self, trial_ids: List[int], group: str) -> List[TrialMetrics]:
        return self.iter_trials_metrics(trial_ids, group)

    def stream_trials_training_metrics(self, trial_ids: List[int]) -> List[TrialMetrics]:
        return self.iter_trials_metrics(trial_ids, "training")

    def stream_trials_validation_metrics(self, trial_ids: List[int]) -> List[TrialMetrics]:
        return self.iter_trials_metrics(trial_ids, "validation")


# ----------------------------------------------------------------------------- test_one_batch
def test_one_batch(trial_class: Type[Any], config: Optional[Dict[str, Any]] = None) -> None:
    """Run one training batch, one validation batch and a checkpoint of a ``PyTorchTrial`` (or
    ``DeepSpeedTrial``) locally in test mode (reference ``experimental/_native.py:test_one_batch``):
    the quickest check that a trial definition works before submitting it."""
    from determined_amd import pytorch

    config = {**(config or {}), "scheduling_unit": 1}
    logger.info("Running a minimal test experiment locally")
    try:
        from determined_amd.pytorch import deepspeed as ds

        is_ds = issubclass(trial_class, ds.DeepSpeedTrial)
    except ImportError:  # pragma: no cover
        is_ds = False
    init = pytorch.deepspeed.init if is_ds else pytorch.init
    with init(hparams=config.get("hyperparameters", {}), exp_conf=config,
              enable_tensorboard_logging=False) as ctx:
        trial = trial_class(ctx)
        pytorch.Trainer(trial, ctx).fit(max_length=pytorch.Batch(1), test_mode=True)
    logger.info("The test experiment passed.")
