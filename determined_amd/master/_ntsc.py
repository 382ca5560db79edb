"""Notebooks, shells, TensorBoards and commands ("NTSC" tasks) plus master config/log routes
(reference: ``master/internal/command/*``, ``api_notebook.go``, ``api_shell.go``,
``api_tensorboard.go``, ``api_command.go``, ``api_master.go`` GetMasterConfig / MasterLogs).

Every NTSC task is a generic command allocation (``Master.create_command``) whose entrypoint is
one of the ``determined_amd.exec`` task programs; once running, a task reports where it lives
(``POST /api/v1/tasks/<id>/proxy``) and the CLI reads that back.
"""

import collections
import logging
import secrets
import sys
import time
from typing import Any, Callable, Deque, Dict, List, Optional

KINDS = {"notebooks": "NOTEBOOK", "shells": "SHELL", "tensorboards": "TENSORBOARD", "commands": "COMMAND"}


class _RingHandler(logging.Handler):
    """Keeps the master's last log records for ``GET /api/v1/master/logs``."""

    def __init__(self, cap: int = 5000) -> None:
        super().__init__(logging.INFO)
        self.records: Deque[Dict[str, Any]] = collections.deque(maxlen=cap)
        self.seq = 0

    def emit(self, record: logging.LogRecord) -> None:
        self.seq += 1
        self.records.append({"id": self.seq, "ts": record.created, "level": record.levelname,
                             "logger": record.name, "message": record.getMessage()})


_RING = _RingHandler()
logging.getLogger("determined_amd").addHandler(_RING)


# the expconf sections a command / notebook / shell / tensorboard container honours (reference
# CommandConfig: environment, bind_mounts, resources; master/pkg/model/command_config.go)
TASK_CONFIG_KEYS = ("environment", "bind_mounts", "resources")


def task_config(b: Dict[str, Any], template: Optional[Dict[str, Any]] = None) -> Optional[Dict[str, Any]]:
    """The request's ``config`` (over its template's) restricted to TASK_CONFIG_KEYS; None if empty."""
    out: Dict[str, Any] = {}
    for src in (template or {}, b.get("config") or {}):
        for k in TASK_CONFIG_KEYS:
            if src.get(k) is not None:
                out[k] = src[k]
    return out or None


def task_command(kind: str, b: Dict[str, Any]) -> List[str]:
    py = [sys.executable, "-m"]
    if kind == "TENSORBOARD":
        ids = ",".join(str(int(x)) for x in b.get("experiment_ids") or [])
        tids = ",".join(str(int(x)) for x in b.get("trial_ids") or [])
        if not ids and not tids:
            raise ValueError("a tensorboard needs experiment_ids or trial_ids")
        return py + ["determined_amd.exec.tensorboard", "--experiment-ids", ids, "--trial-ids", tids]
    if kind == "SHELL":
        return py + ["determined_amd.exec.shell", "--idle-timeout", str(float(b.get("idle_timeout", 0)))]
    if kind == "NOTEBOOK":
        return py + ["determined_amd.exec.notebook"]
    cmd = b.get("command") or b.get("entrypoint")
    if not cmd:
        raise ValueError("a command needs 'command'")
    return cmd


def add_ntsc_routes(route: Callable[[str, str], Callable], m: Any) -> None:
    for plural, kind in KINDS.items():
        if kind == "COMMAND":
            continue  # POST /api/v1/commands is the generic route in _server

        def make_create(kind=kind):
            def create(q, b):
                env = dict(b.get("env") or {})
                if kind == "NOTEBOOK":
                    env["DET_NOTEBOOK_TOKEN"] = secrets.token_hex(16)
                try:
                    cmd = task_command(kind, b)
                except ValueError as e:
                    from determined_amd.master._server import HTTPError

                    raise HTTPError(400, str(e))
                tid = m.create_command(cmd, int(b.get("slots", 0)), env, kind, b.get("workdir_b64"),
                                       b.get("resource_pool"), b.get("priority"), task_config=task_config(b))
                return {"task_id": tid, "type": kind}
            return create

        route("POST", f"/api/v1/{plural}")(make_create())

    for plural, kind in KINDS.items():
        def make_list(kind=kind):
            def lst(q, b):
                from determined_amd.master._server import public_task

                rows = [public_task(r) for r in m.db.all("SELECT * FROM tasks WHERE type=? ORDER BY start_time", [kind])]
                return {"tasks": rows}
            return lst

        route("GET", f"/api/v1/{plural}")(make_list())

    @route("GET", "/api/v1/master/config")
    def master_config(q, b):
        m.iam.require("view")
        import logging as _logging

        return {"config": {"scheduler": {"type": m.policy, "fitting_policy": getattr(m, "fit", None)},
                           "auth": m.iam.mode, "master_url": m.master_url, "cluster_id": m.cluster_id,
                           "db": m.db.path, "log_retention_days": None,
                           "resource_pools": m.sched.summary(),
                           "resource_manager": {"default_compute_resource_pool": m.sched.default_compute,
                                                "default_aux_resource_pool": m.sched.default_aux},
                           "log": {"level": _logging.getLevelName(
                               _logging.getLogger("determined_amd").getEffectiveLevel()).lower()}}}

    @route("PATCH", "/api/v1/master/config")
    def master_config_set(q, b):
        """Runtime-mutable master settings (reference ``det master config set --log.level``)."""
        import logging as _logging

        m.iam.require("admin_cluster")
        level = (b.get("log") or {}).get("level")
        if level is not None:
            lv = _logging.getLevelName(str(level).upper())
            if not isinstance(lv, int):
                raise ValueError(f"unknown log level {level!r}")
            _logging.getLogger("determined_amd").setLevel(lv)
        return master_config(q, b)

    @route("POST", "/api/v1/tasks/cleanup-logs")
    def cleanup_logs(q, b):
        """Apply the log retention policies now (reference ``det task cleanup-logs``)."""
        m.iam.require("admin_cluster")
        return {"removed": m.cleanup_logs()}

    @route("GET", "/api/v1/master/logs")
    def master_logs(q, b):
        m.iam.require("admin_cluster")
        after = int(q.get("after", 0))
        limit = int(q.get("limit", 1000))
        recs = [r for r in list(_RING.records) if r["id"] > after]
        return {"logs": recs[-limit:], "now": time.time()}
