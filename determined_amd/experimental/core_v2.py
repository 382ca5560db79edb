"""Core API v2 (reference: ``harness/determined/experimental/core_v2``).

One call covers both modes:

* managed (launched by the master as a TRIAL): identical to ``core.init()``;
* unmanaged (any script anywhere that can reach the master): an *unmanaged* experiment and
  trial are created (or found again through ``external_experiment_id`` /
  ``external_trial_id`` for resumption and multi-trial grouping) and the script reports
  metrics and checkpoints to them; the searcher is a single local operation and there is no
  preemption.

.. code-block:: python

    from determined_amd.experimental import core_v2
    core_v2.init(defaults=core_v2.DefaultConfig(name="my-run", hparams={"lr": 0.1}),
                 unmanaged=core_v2.UnmanagedConfig(external_experiment_id="run-7"))
    core_v2.train.report_training_metrics(steps_completed=10, metrics={"loss": 0.3})
    core_v2.close()

The singleton style exposes ``core_v2.train``, ``checkpoint``, ``distributed``, ``preempt``,
``searcher`` and ``info`` after ``init()``; ``init_context()`` returns the context instead.
"""

import atexit
import dataclasses
import os
import uuid
from typing import Any, Dict, List, Optional, Union

from determined_amd import core
from determined_amd._info import ClusterInfo, TrialInfo, get_cluster_info
from determined_amd.common.api import Session


@dataclasses.dataclass
class DefaultConfig:
    name: Optional[str] = None
    hparams: Optional[Dict[str, Any]] = None
    data: Optional[Dict[str, Any]] = None
    description: Optional[str] = None
    labels: Optional[List[str]] = None
    checkpoint_storage: Optional[Union[str, Dict[str, Any]]] = None
    searcher: Optional[Dict[str, Any]] = None


@dataclasses.dataclass
class UnmanagedConfig:
    workspace: Optional[str] = None
    project: Optional[str] = None
    external_experiment_id: Optional[str] = None
    external_trial_id: Optional[str] = None


_context: Optional[core.Context] = None
_atexit_registered = False
train: Any = None
checkpoint: Any = None
distributed: Any = None
preempt: Any = None
searcher: Any = None
info: Any = None


def _default_storage() -> Dict[str, Any]:
    base = os.environ.get("DET_LOCAL_CHECKPOINT_DIR", os.path.expanduser("~/.local/share/determined_amd"))
    return {"type": "shared_fs", "host_path": base}


def _unmanaged_info(session: Session, defaults: DefaultConfig, unmanaged: UnmanagedConfig,
                    dist: Optional[core.DistributedContext],
                    checkpoint_storage: Optional[Union[str, Dict[str, Any]]]) -> ClusterInfo:
    if unmanaged.external_trial_id and not unmanaged.external_experiment_id:
        raise ValueError("external_trial_id requires external_experiment_id")
    storage_cfg = checkpoint_storage or defaults.checkpoint_storage or _default_storage()
    if isinstance(storage_cfg, str):
        storage_cfg = {"type": "shared_fs", "host_path": storage_cfg}
    cfg: Dict[str, Any] = {
        "name": defaults.name or f"unmanaged-{uuid.uuid4().hex[:8]}",
        "data": defaults.data or {},
        "description": defaults.description or "",
        "labels": defaults.labels or [],
        "searcher": defaults.searcher or {"name": "single", "metric": "unmanaged", "max_length": {"batches": 10**8}},
        "checkpoint_storage": storage_cfg,
        "hyperparameters": {k: {"type": "const", "val": v} for k, v in (defaults.hparams or {}).items()},
    }
    if unmanaged.workspace:
        cfg["workspace"] = unmanaged.workspace
    if unmanaged.project:
        cfg["project"] = unmanaged.project
    rank = dist.rank if dist is not None else 0

    def create() -> Dict[str, Any]:
        exp = session.post("/api/v1/unmanaged/experiments",
                           {"config": cfg, "external_experiment_id": unmanaged.external_experiment_id})["experiment"]
        tr = session.post(f"/api/v1/unmanaged/experiments/{exp['id']}/trials",
                          {"hparams": defaults.hparams or {}, "external_trial_id": unmanaged.external_trial_id})
        full = session.get(f"/api/v1/experiments/{exp['id']}")["config"]
        return {"exp_id": exp["id"], "trial": tr, "config": full}

    res = create() if rank == 0 else None
    if dist is not None and dist.size > 1:
        res = dist.broadcast(res)
    assert res is not None
    tid = int(res["trial"]["trial_id"])
    trial = TrialInfo(trial_id=tid, experiment_id=int(res["exp_id"]), trial_seed=0, hparams=defaults.hparams or {},
                      config=res["config"], steps_completed=int(res["trial"].get("steps_completed") or 0),
                      trial_run_id=0)
    return ClusterInfo(master_url=session.master_url, cluster_id="unmanaged", agent_id="unmanaged",
                       slot_ids=[], task_id=f"trial-{tid}", allocation_id=f"unmanaged-{tid}",
                       session_token=session.token or "", task_type="TRIAL", container_addrs=["127.0.0.1"],
                       container_rank=0, latest_checkpoint=res["trial"].get("latest_checkpoint"), trial=trial)


def init_context(*, defaults: Optional[DefaultConfig] = None, unmanaged: Optional[UnmanagedConfig] = None,
                 master: Optional[str] = None, distributed: Optional[core.DistributedContext] = None,
                 checkpoint_storage: Optional[Union[str, Dict[str, Any]]] = None,
                 preempt_mode: core.PreemptMode = core.PreemptMode.WorkersAskChief,
                 tensorboard_mode: Any = None) -> core.Context:
    managed = get_cluster_info()
    if managed is not None and managed.task_type == "TRIAL":
        return core.init(distributed=distributed, checkpoint_storage=checkpoint_storage, preempt_mode=preempt_mode,
                         tensorboard_mode=tensorboard_mode)
    if defaults is None:
        raise NotImplementedError("either specify `defaults`, or run as a managed experiment")
    session = Session(master or os.environ.get("DET_MASTER", "http://127.0.0.1:8080"))
    ci = _unmanaged_info(session, defaults, unmanaged or UnmanagedConfig(), distributed, checkpoint_storage)
    ctx = core.init(distributed=distributed, checkpoint_storage=checkpoint_storage, preempt_mode=preempt_mode,
                    tensorboard_mode=tensorboard_mode, _info=ci, _unmanaged=True,
                    _heartbeat_interval=float(os.environ.get("DET_UNMANAGED_HEARTBEAT_S", "60")))
    ctx._unmanaged_session = session  # type: ignore[attr-defined]
    return ctx


def _set_globals(ctx: Optional[core.Context]) -> None:
    global train, checkpoint, distributed, preempt, searcher, info
    train = ctx.train if ctx else None
    checkpoint = ctx.checkpoint if ctx else None
    distributed = ctx.distributed if ctx else None
    preempt = ctx.preempt if ctx else None
    searcher = ctx.searcher if ctx else None
    info = ctx.info if ctx else None


def init(**kwargs: Any) -> None:
    """Singleton-style ``init_context``; ``close()`` (also registered at exit) finishes the trial."""
    global _context, _atexit_registered
    if _context is not None:
        close()
    _context = init_context(**kwargs)
    _context.__enter__()
    _set_globals(_context)
    if not _atexit_registered:
        atexit.register(close)
        _atexit_registered = True


def close(state: str = "COMPLETED") -> None:
    """Finish the trial.  Unmanaged: the chief's heartbeat reports the final state -- ``state``, or ERROR
    when the process is exiting on an uncaught exception / a non-zero ``sys.exit`` (``core/_heartbeat.py``)."""
    global _context
    if _context is None:
        return
    ctx, _context = _context, None
    try:
        hb = getattr(ctx, "_heartbeat", None)
        if hb is not None:
            hb.requested_state = state
    finally:
        ctx.__exit__(None, None, None)
        _set_globals(None)


def url_reverse_webui_exp_view() -> str:
    if info is None:
        raise RuntimeError("core_v2.init() has not been called")
    return f"{info.master_url}/det/experiments/{info.trial.experiment_id}"
