"""Master REST API (reference: ``master/internal/api_*.go`` behind grpc-gateway).

JSON over HTTP on a threaded stdlib server; routes mirror the reference's ``/api/v1`` paths the
harness and CLI use.  Long-polling endpoints (agent work, preemption signals, searcher events)
block on the master's condition variable.
"""

import base64
import json
import pathlib
import logging
import re
import threading
import time
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Callable, Dict, List, Optional, Tuple

from determined_amd import __version__
from determined_amd.config import InvalidConfig
from determined_amd.master._iam import AuthError, _public_user
from determined_amd.master._iam_routes import add_iam_routes
from determined_amd.master._ntsc import add_ntsc_routes, task_config
from determined_amd.master._exp_routes import add_exp_routes
from determined_amd.master._runs_routes import add_runs_routes
from determined_amd.master._webui import add_webui_routes
from determined_amd.master._core import Master

logger = logging.getLogger("determined_amd.master")

Route = Tuple[str, "re.Pattern[str]", Callable[..., Any]]


def _ts(v: Any, default: float) -> float:
    """A query timestamp: epoch seconds or ISO-8601 (``2024-01-31T12:00:00Z``)."""
    if v in (None, ""):
        return default
    try:
        return float(v)
    except ValueError:
        import datetime

        return datetime.datetime.fromisoformat(str(v).replace("Z", "+00:00")).timestamp()


class HTTPError(Exception):
    def __init__(self, status: int, message: str) -> None:
        super().__init__(message)
        self.status = status
        self.message = message


def _guard_exp(m: Master, eid: Any, perm: str) -> Dict[str, Any]:
    row = m.db.one("SELECT id, owner, workspace FROM experiments WHERE id=?", [int(eid)])
    if row is None:
        raise HTTPError(404, f"experiment {eid} not found")
    sc = m.iam.experiment_scope(row)
    m.iam.require(perm, sc["workspace_id"], sc["owner_id"])
    return row


def deep_merge(primary: Any, fallback: Any) -> Any:
    """``primary`` with the keys it lacks filled from ``fallback``, recursively through dicts
    (reference ``schemas.Merge``: the experiment's own settings win over the template's)."""
    if isinstance(primary, dict) and isinstance(fallback, dict):
        out = dict(fallback)
        for k, v in primary.items():
            out[k] = deep_merge(v, fallback[k]) if k in fallback else v
        return out
    return primary


def merge_template(m: Master, cfg: Dict[str, Any], name: str) -> Dict[str, Any]:
    row = m.db.one("SELECT * FROM templates WHERE name=?", [name])
    if row is None:
        raise HTTPError(404, f"template {name} not found")
    tcfg = row["config"]
    if isinstance(tcfg, (str, bytes)):
        tcfg = json.loads(tcfg)
    return deep_merge(cfg, tcfg or {})


def _exp_summary(m: Master, row: Dict[str, Any]) -> Dict[str, Any]:
    cfg = row.get("config") or {}
    n = m.db.one("SELECT COUNT(*) AS n FROM trials WHERE experiment_id=?", [row["id"]])
    return {
        "id": row["id"], "name": row.get("name"), "state": row["state"], "archived": bool(row.get("archived")),
        "progress": row.get("progress") or 0.0, "start_time": row.get("start_time"), "end_time": row.get("end_time"),
        "description": row.get("description"), "labels": row.get("labels") or [], "owner": row.get("owner"),
        "project": row.get("project"), "workspace": row.get("workspace"), "num_trials": n["n"] if n else 0,
        "searcher_type": cfg.get("searcher", {}).get("name"), "parent_id": row.get("parent_id"),
        "unmanaged": bool(row.get("unmanaged")),
    }


def _trial_summary(m: Master, t: Dict[str, Any]) -> Dict[str, Any]:
    lv = m.db.one("SELECT steps_completed, metrics FROM metrics WHERE trial_id=? AND group_name='validation' "
                  "ORDER BY id DESC LIMIT 1", [t["id"]])
    lt = m.db.one("SELECT steps_completed, metrics FROM metrics WHERE trial_id=? AND group_name='training' "
                  "ORDER BY id DESC LIMIT 1", [t["id"]])
    return {
        "id": t["id"], "experiment_id": t["experiment_id"], "request_id": t["request_id"], "state": t["state"],
        "hparams": t["hparams"], "seed": t["seed"], "restarts": t["restarts"], "run_id": t["run_id"],
        "start_time": t["start_time"], "end_time": t["end_time"], "latest_checkpoint": t["latest_checkpoint"],
        "total_batches": t["total_batches"], "searcher_metric": t["searcher_metric"],
        "best_validation": t["best_validation"], "runner_state": t.get("runner_state"),
        "latest_validation": lv, "latest_training": lt, "task_id": f"trial-{t['id']}",
    }


def build_routes(m: Master) -> List[Route]:
    routes: List[Route] = []

    def route(method: str, pattern: str):
        def deco(fn):
            routes.append((method, re.compile("^" + pattern + "$"), fn))
            return fn

        return deco

    # ---------------------------------------------------------------- master
    @route("GET", "/api/v1/master")
    def master_info(q, b):
        return {"version": __version__, "cluster_id": m.cluster_id, "master_id": m.cluster_id,
                "cluster_name": "determined_amd", "scheduler": m.policy,
                "total_slots": m.sched.total_slots, "used_slots": m.sched.used_slots}

    @route("GET", "/api/v1/me")
    def me(q, b):
        return {"user": _public_user(m.iam.current())}

    @route("POST", "/api/v1/auth/login")
    def login(q, b):
        return m.iam.login(b.get("username", "determined"), b.get("password", ""))

    add_iam_routes(route, m)

    # ---------------------------------------------------------------- experiments
    @route("POST", "/api/v1/experiments")
    def create_exp(q, b):
        md = base64.b64decode(b["model_def"]) if b.get("model_def") else None
        cfg0 = b["config"] if isinstance(b.get("config"), dict) else {}
        if b.get("template"):  # reference core_experiment.go: schemas.Merge(config, template)
            cfg0 = merge_template(m, cfg0, b["template"])
        if b.get("project_id") is not None:  # place the experiment in this project
            proj = m.db.one("SELECT * FROM projects WHERE id=?", [int(b["project_id"])])
            if proj is None:
                raise HTTPError(404, f"project {b['project_id']} not found")
            ws = m.db.one("SELECT name FROM workspaces WHERE id=?", [proj["workspace_id"]])
            cfg0 = dict(cfg0, workspace=ws["name"], project=proj["name"])
        m.iam.resolve_target(cfg0)
        try:
            eid = m.create_experiment(cfg0 if isinstance(b.get("config"), dict) else b["config"], md,
                                      activate=b.get("activate", True),
                                      parent_id=b.get("parent_id"), unmanaged=bool(b.get("unmanaged")))
        except InvalidConfig as e:
            raise HTTPError(400, str(e))
        return {"experiment": _exp_summary(m, m.db.one("SELECT * FROM experiments WHERE id=?", [eid]))}

    @route("POST", "/api/v1/unmanaged/experiments")
    def create_unmanaged_exp(q, b):
        try:
            eid = m.create_unmanaged_experiment(b["config"], b.get("external_experiment_id"))
        except InvalidConfig as e:
            raise HTTPError(400, str(e))
        return {"experiment": _exp_summary(m, m.db.one("SELECT * FROM experiments WHERE id=?", [eid]))}

    @route("POST", r"/api/v1/unmanaged/experiments/(\d+)/trials")
    def create_unmanaged_trial(q, b, eid):
        return m.create_unmanaged_trial(int(eid), b.get("hparams") or {}, b.get("external_trial_id"))

    @route("POST", r"/api/v1/unmanaged/trials/(\d+)/close")
    def close_unmanaged_trial(q, b, tid):
        m.close_unmanaged_trial(int(tid), b.get("state", "COMPLETED"))
        return {}

    @route("GET", "/api/v1/experiments")
    def list_exps(q, b):
        rows = m.db.all("SELECT * FROM experiments WHERE state!='DELETED' ORDER BY id")
        if q.get("workspace"):
            rows = [r for r in rows if r.get("workspace") == q["workspace"]]
        if q.get("project"):
            rows = [r for r in rows if r.get("project") == q["project"]]
        if q.get("user"):
            rows = [r for r in rows if r.get("owner") == q["user"]]
        if q.get("archived") in ("false", "0"):
            rows = [r for r in rows if not r["archived"]]
        return {"experiments": [_exp_summary(m, r) for r in rows]}

    @route("GET", r"/api/v1/experiments/(\d+)")
    def get_exp(q, b, eid):
        row = m.db.one("SELECT * FROM experiments WHERE id=?", [int(eid)])
        if row is None:
            raise HTTPError(404, f"experiment {eid} not found")
        return {"experiment": _exp_summary(m, row), "config": row["config"]}

    @route("GET", r"/api/v1/experiments/(\d+)/model_def")
    def get_model_def(q, b, eid):
        row = m.db.one("SELECT model_def FROM experiments WHERE id=?", [int(eid)])
        if row is None:
            raise HTTPError(404, "not found")
        md = row["model_def"]
        return {"b64_tgz": base64.b64encode(md).decode() if md else None}

    for action, fn_name in (("pause", "pause_experiment"), ("activate", "activate_experiment"),
                            ("kill", "kill_experiment"), ("cancel", "kill_experiment")):
        def make(fn_name=fn_name):
            def handler(q, b, eid):
                _guard_exp(m, eid, "edit")
                getattr(m, fn_name)(int(eid))
                return {}
            return handler

        routes.append(("POST", re.compile(rf"^/api/v1/experiments/(\d+)/{action}$"), make()))

    @route("POST", r"/api/v1/experiments/(\d+)/archive")
    def archive(q, b, eid):
        _guard_exp(m, eid, "edit")
        m.archive_experiment(int(eid), True)
        return {}

    @route("POST", r"/api/v1/experiments/(\d+)/unarchive")
    def unarchive(q, b, eid):
        _guard_exp(m, eid, "edit")
        m.archive_experiment(int(eid), False)
        return {}

    @route("DELETE", r"/api/v1/experiments/(\d+)")
    def delete_exp(q, b, eid):
        _guard_exp(m, eid, "edit")
        try:
            m.delete_experiment(int(eid))
        except ValueError as e:
            raise HTTPError(400, str(e))
        return {}

    @route("PATCH", r"/api/v1/experiments/(\d+)")
    def patch_exp(q, b, eid):
        _guard_exp(m, eid, "edit")
        cols = {k: v for k, v in b.items() if k in ("name", "description", "notes", "labels")}
        m.db.update("experiments", "id", int(eid), **cols)
        return {}

    @route("GET", r"/api/v1/experiments/(\d+)/trials")
    def exp_trials(q, b, eid):
        rows = m.db.all("SELECT * FROM trials WHERE experiment_id=? ORDER BY id", [int(eid)])
        return {"trials": [_trial_summary(m, t) for t in rows]}

    @route("GET", r"/api/v1/experiments/(\d+)/checkpoints")
    def exp_ckpts(q, b, eid):
        rows = m.db.all("SELECT * FROM checkpoints WHERE experiment_id=? ORDER BY report_time", [int(eid)])
        return {"checkpoints": rows}

    @route("GET", r"/api/v1/experiments/(\d+)/searcher/best_searcher_validation_metric")
    def best_val(q, b, eid):
        v = m.best_searcher_validation(int(eid))
        if v is None:
            raise HTTPError(404, "no validations yet")
        return {"metric": v}

    @route("GET", r"/api/v1/experiments/(\d+)/searcher_events")
    def searcher_events(q, b, eid):
        return {"events": m.get_searcher_events(int(eid), float(q.get("timeout_seconds", 0)))}

    @route("POST", r"/api/v1/experiments/(\d+)/searcher_operations")
    def searcher_ops(q, b, eid):
        m.post_searcher_operations(int(eid), b.get("operations", []), int(b.get("triggered_by_event", 0)))
        return {}

    @route("POST", r"/api/v1/experiments/(\d+)/gc")
    def exp_gc(q, b, eid):
        return {"deleted": m.gc_experiment_checkpoints(int(eid))}

    # ---------------------------------------------------------------- trials
    @route("GET", r"/api/v1/trials/(\d+)")
    def get_trial(q, b, tid):
        t = m.db.one("SELECT * FROM trials WHERE id=?", [int(tid)])
        if t is None:
            raise HTTPError(404, f"trial {tid} not found")
        return {"trial": _trial_summary(m, t)}

    @route("GET", r"/api/v1/trials/(\d+)/searcher/operation")
    def trial_op(q, b, tid):
        try:
            return m.get_searcher_op(int(tid))
        except KeyError as e:
            raise HTTPError(404, str(e))

    @route("POST", r"/api/v1/trials/(\d+)/searcher/completed_operation")
    def trial_op_done(q, b, tid):
        try:
            m.complete_searcher_op(int(tid), int(b["op"]["length"]), b["searcher_metric"])
        except ValueError as e:
            raise HTTPError(400, str(e))
        return {}

    @route("POST", r"/api/v1/trials/(\d+)/progress")
    def trial_progress(q, b, tid):
        m.report_progress(int(tid), float(b.get("progress", 0.0)))
        return {}

    @route("POST", r"/api/v1/trials/(\d+)/metrics")
    def trial_metrics(q, b, tid):
        m.report_metrics(int(tid), b)
        return {}

    @route("GET", r"/api/v1/trials/(\d+)/metrics")
    def get_trial_metrics(q, b, tid):
        grp = q.get("group")
        rows = m.db.all("SELECT group_name, steps_completed, metrics, trial_run_id, ts FROM metrics WHERE trial_id=? "
                        + ("AND group_name=? " if grp else "") + "ORDER BY id", [int(tid)] + ([grp] if grp else []))
        return {"metrics": rows}

    # ---------------------------------------------------------------- trial source info (reference
    # api_trials.go ReportTrialSourceInfo / GetTrialMetricsByCheckpoint / ...ByModelVersion): a task
    # that runs a checkpoint (batch inference) links itself to it, and the checkpoint's / model
    # version's metrics are the metrics those tasks reported.
    @route("POST", "/api/v1/trial-source-info")
    def report_source_info(q, b):
        info = b.get("trial_source_info") or b
        tid = int(info["trial_id"])
        if m.db.one("SELECT id FROM trials WHERE id=?", [tid]) is None:
            raise HTTPError(404, f"trial {tid} not found")
        uuid_ = info["checkpoint_uuid"]
        if m.db.one("SELECT uuid FROM checkpoints WHERE uuid=?", [uuid_]) is None:
            raise HTTPError(404, f"checkpoint {uuid_} not found")
        m.db.execute("INSERT OR REPLACE INTO trial_source_infos (trial_id, checkpoint_uuid, source_type, model_id, "
                     "model_version) VALUES (?,?,?,?,?)",
                     [tid, uuid_, info.get("trial_source_info_type", "INFERENCE"), info.get("model_id"),
                      info.get("model_version")])
        return {"trial_id": tid, "checkpoint_uuid": uuid_}

    def _source_metrics(where: str, args: List[Any], q: Dict[str, str]) -> Dict[str, Any]:
        kind = q.get("trial_source_info_type", "INFERENCE")
        grp = q.get("group") or q.get("metric_group")
        tids = [int(r["trial_id"]) for r in m.db.all(
            f"SELECT DISTINCT trial_id FROM trial_source_infos WHERE {where} AND source_type=? ORDER BY trial_id",
            args + [kind])]
        out = []
        for tid in tids:
            rows = m.db.all("SELECT group_name, steps_completed, metrics, trial_run_id, ts FROM metrics WHERE "
                            "trial_id=? " + ("AND group_name=? " if grp else "") + "ORDER BY id",
                            [tid] + ([grp] if grp else []))
            out.extend(dict(r, trial_id=tid) for r in rows)
        return {"metrics": out}

    @route("GET", r"/api/v1/checkpoints/([^/]+)/metrics")
    def checkpoint_metrics(q, b, uuid_):
        return _source_metrics("checkpoint_uuid=?", [uuid_], q)

    @route("GET", r"/api/v1/models/([^/]+)/versions/(\d+)/metrics")
    def model_version_metrics(q, b, name, ver):
        mod = m.db.one("SELECT id FROM models WHERE name=? OR CAST(id AS TEXT)=?", [name, name])
        if mod is None:
            raise HTTPError(404, f"model {name} not found")
        return _source_metrics("model_id=? AND model_version=?", [int(mod["id"]), int(ver)], q)

    @route("POST", r"/api/v1/trials/(\d+)/early_exit")
    def trial_early_exit(q, b, tid):
        try:
            m.early_exit(int(tid), b.get("reason", ""))
        except ValueError as e:
            raise HTTPError(400, str(e))
        return {}

    @route("POST", r"/api/v1/trials/(\d+)/runner/metadata")
    def trial_runner(q, b, tid):
        m.db.update("trials", "id", int(tid), runner_state=b.get("state", ""))
        return {}

    @route("POST", r"/api/v1/trials/(\d+)/kill")
    def trial_kill(q, b, tid):
        with m.lock:
            _, tr = m._trial(int(tid))
            if tr.allocation is not None:
                m._kill_allocation(tr.allocation)
        return {}

    @route("GET", r"/api/v1/trials/(\d+)/checkpoints")
    def trial_ckpts(q, b, tid):
        return {"checkpoints": m.db.all("SELECT * FROM checkpoints WHERE trial_id=? ORDER BY report_time", [int(tid)])}

    # ---------------------------------------------------------------- checkpoints
    @route("POST", "/api/v1/checkpoints")
    def report_ckpt(q, b):
        m.report_checkpoint(b)
        return {}

    @route("GET", r"/api/v1/checkpoints/([0-9a-f\-]+)")
    def get_ckpt(q, b, u):
        row = m.db.one("SELECT * FROM checkpoints WHERE uuid=?", [u])
        if row is None:
            raise HTTPError(404, f"checkpoint {u} not found")
        exp = m.db.one("SELECT config FROM experiments WHERE id=?", [row["experiment_id"]]) \
            if row.get("experiment_id") else None
        row["checkpoint_storage"] = (exp or {}).get("config", {}).get("checkpoint_storage") if exp else None
        return {"checkpoint": row}

    @route("GET", r"/api/v1/checkpoints/([0-9a-f\-]+)/download")
    def download_ckpt(q, b, u):
        """The checkpoint's files as one tar.gz streamed by the master (reference ``DownloadMode.MASTER``,
        ``GET /checkpoints/<uuid>`` with ``Accept: application/gzip``): for clients that cannot reach the
        checkpoint storage themselves.  The master reads it through the experiment's storage config."""
        import io
        import tarfile
        import tempfile

        from determined_amd import storage as det_storage

        row = m.db.one("SELECT * FROM checkpoints WHERE uuid=?", [u])
        if row is None:
            raise HTTPError(404, f"checkpoint {u} not found")
        if row.get("state") == "DELETED":
            raise HTTPError(409, f"checkpoint {u} was deleted")
        exp = m.db.one("SELECT id, config FROM experiments WHERE id=?", [row["experiment_id"]]) \
            if row.get("experiment_id") else None
        if exp is None:
            raise HTTPError(404, f"checkpoint {u} has no experiment storage configuration")
        _guard_exp(m, exp["id"], "view")
        sm = det_storage.build((exp.get("config") or {}).get("checkpoint_storage"))
        buf = io.BytesIO()
        with tempfile.TemporaryDirectory() as td:
            try:
                sm.download(src=u, dst=td)
            except (OSError, RuntimeError) as e:
                raise HTTPError(502, f"master could not read checkpoint {u} from storage: {e}")
            with tarfile.open(fileobj=buf, mode="w:gz") as tf:
                for f in sorted(pathlib.Path(td).rglob("*")):
                    tf.add(str(f), arcname=str(f.relative_to(td)), recursive=False)
        return _Raw(buf.getvalue(), "application/gzip")

    @route("PATCH", r"/api/v1/checkpoints/([0-9a-f\-]+)")
    def patch_ckpt(q, b, u):
        if m.db.one("SELECT uuid FROM checkpoints WHERE uuid=?", [u]) is None:
            raise HTTPError(404, f"checkpoint {u} not found")
        if "metadata" in b:
            m.db.update("checkpoints", "uuid", u, metadata=b["metadata"])
        if "resources" in b:  # partial GC (exec/gc_checkpoints.py --globs) reports what is left
            m.db.update("checkpoints", "uuid", u, resources=b["resources"])
        if b.get("state") in ("PARTIALLY_DELETED", "DELETED"):
            m.db.update("checkpoints", "uuid", u, state=b["state"])
        return {}

    @route("DELETE", r"/api/v1/checkpoints/([0-9a-f\-]+)")
    def del_ckpt(q, b, u):
        m.delete_checkpoints([u])
        return {}

    # ---------------------------------------------------------------- allocations
    @route("GET", r"/api/v1/allocations/([^/]+)/signals/preemption")
    def preempt(q, b, aid):
        return {"preempt": m.preemption_signal(aid, float(q.get("timeout_seconds", 0)))}

    @route("POST", r"/api/v1/allocations/([^/]+)/signals/ack_preemption")
    def ack(q, b, aid):
        m.ack_preemption(aid)
        return {}

    @route("POST", r"/api/v1/allocations/([^/]+)/all_gather")
    def all_gather(q, b, aid):
        return {"data": m.allocation_all_gather(aid, str(b["request_uuid"]), int(b["num_peers"]), b.get("data"),
                                                b.get("rank"), float(b.get("timeout_seconds", 600)))}

    @route("GET", "/api/v1/stream")
    def stream(q, b):
        ents = [e for e in q.get("entities", "").split(",") if e]
        return m.stream(int(q.get("since", 0)), min(float(q.get("timeout_seconds", 0)), 60.0), ents or None,
                        q.get("epoch") or None)

    @route("GET", "/api/v1/allocations")
    def allocs(q, b):
        return {"allocations": [a.to_dict() for a in m.allocations.values() if a.state != "TERMINATED"]}

    # ---------------------------------------------------------------- logs / tasks
    @route("POST", "/api/v1/task/logs")
    def post_logs(q, b):
        m.add_logs(b["task_id"], b.get("logs", []), b.get("allocation_id"))
        return {}

    @route("GET", r"/api/v1/tasks/([^/]+)/logs")
    def task_logs(q, b, task_id):
        return {"logs": m.get_logs(task_id, int(q.get("after", 0)), int(q.get("limit", 10000)))}

    @route("POST", "/api/v1/commands")
    def create_cmd(q, b):
        tcfg = None
        if b.get("template"):  # reference api_command.go: the template's config fills what the request lacks
            tcfg = merge_template(m, {}, b["template"])
            res = tcfg.get("resources") or {}
            b = dict(b)
            if b.get("slots") is None:
                b["slots"] = res.get("slots", 0)
            if b.get("resource_pool") is None:
                b["resource_pool"] = res.get("resource_pool")
            if b.get("priority") is None:
                b["priority"] = res.get("priority")
            env_vars = (tcfg.get("environment") or {}).get("environment_variables") or []
            if isinstance(env_vars, dict):
                env_vars = [f"{k}={v}" for k, v in env_vars.items()]
            env = dict(kv.split("=", 1) for kv in env_vars if "=" in kv)
            env.update(b.get("env") or {})
            b["env"] = env or None
        tid = m.create_command(b["command"], int(b.get("slots") or 0), b.get("env"), b.get("type", "COMMAND"),
                               b.get("workdir_b64"), b.get("resource_pool"), b.get("priority"),
                               task_config=task_config(b, tcfg if b.get("template") else None))
        return {"task_id": tid}

    @route("POST", r"/api/v1/tasks/([^/]+)/(pause|unpause)")
    def task_pause(q, b, task_id, what):
        try:
            (m.pause_task if what == "pause" else m.unpause_task)(task_id)
        except KeyError as e:
            raise HTTPError(404, str(e))
        except ValueError as e:
            raise HTTPError(400, str(e))
        return {}

    @route("GET", "/api/v1/_routes")
    def list_routes(q, b):
        """Every REST route of this master (``det dev bindings list``)."""
        return {"routes": [{"method": meth, "path": rx.pattern.strip("^$")} for meth, rx, _ in routes]}

    @route("POST", r"/api/v1/tasks/([^/]+)/proxy")
    def task_proxy(q, b, task_id):
        """A task registers where its service listens.  Only the cluster identity (the token the
        master hands to its tasks) or an admin may do so, and only to a loopback address or the host
        of a registered agent -- never an arbitrary host (the proxy would otherwise be an SSRF path
        and a way to point another user's notebook at a foreign server)."""
        if m.db.one("SELECT id FROM tasks WHERE id=?", [task_id]) is None:
            raise HTTPError(404, f"task {task_id} not found")
        if not m.iam.current()["admin"]:
            raise HTTPError(403, "only the task itself (cluster token) may register its proxy address")
        host = b.get("host") or "127.0.0.1"
        agent_hosts = {ag.get("host") for ag in m.agents.values()}
        if host not in _LOOPBACK and host not in agent_hosts:
            raise HTTPError(400, f"proxy host {host!r} is neither loopback nor a registered agent's host")
        port = b.get("port")
        if port is not None and not (isinstance(port, int) and 0 < port < 65536):
            raise HTTPError(400, f"invalid proxy port {port!r}")
        px = {"host": host, "port": port, "cwd": b.get("cwd"), "env": b.get("env")}
        if b.get("tunnel"):  # a shell server (exec/shell.py): reached only through /proxy/<task>/_tunnel
            px.update(tunnel=True, shell_key=str(b.get("shell_key") or ""))
        m.db.update("tasks", "id", task_id, proxy=px)
        return {}

    add_ntsc_routes(route, m)
    add_exp_routes(route, m)
    add_runs_routes(route, m)

    @route("GET", "/api/v1/tasks")
    def list_tasks(q, b):
        return {"tasks": [public_task(r) for r in m.db.all("SELECT * FROM tasks ORDER BY start_time")]}

    @route("GET", r"/api/v1/tasks/([^/]+)")
    def get_task(q, b, task_id):
        row = m.db.one("SELECT * FROM tasks WHERE id=?", [task_id])
        if row is None:
            raise HTTPError(404, f"task {task_id} not found")
        return {"task": public_task(row)}

    @route("POST", r"/api/v1/tasks/([^/]+)/kill")
    def kill_task(q, b, task_id):
        m.kill_task(task_id)
        return {}

    # ---------------------------------------------------------------- agents
    @route("POST", "/api/v1/agents/register")
    def reg_agent(q, b):
        return m.register_agent(b["agent_id"], int(b["slots"]), b.get("host", "127.0.0.1"), b.get("devices"),
                                bool(b.get("gpu")), b.get("label", ""), b.get("resource_pool"), b.get("running"))

    @route("GET", r"/api/v1/agents/([^/]+)/work")
    def agent_work(q, b, agent_id):
        try:
            return {"commands": m.agent_poll(agent_id, float(q.get("timeout_seconds", 10)))}
        except KeyError as e:
            raise HTTPError(404, str(e))

    @route("POST", r"/api/v1/agents/([^/]+)/events")
    def agent_ev(q, b, agent_id):
        m.agent_event(agent_id, b)
        return {}

    @route("GET", "/api/v1/agents")
    def list_agents(q, b):
        sa = m.sched.agents()
        out = []
        for aid, ag in m.agents.items():
            owners = sa.get(aid, {}).get("slot_owner", [])
            out.append({"id": aid, "host": ag["host"], "slots": ag["slots"], "devices": ag["devices"],
                        "gpu": ag["gpu"], "enabled": ag["enabled"], "label": ag["label"],
                        "resource_pool": ag.get("resource_pool", m.sched.default_compute),
                        "slot_owner": owners, "used_slots": sum(1 for o in owners if o),
                        "disabled_slots": list(sa.get(aid, {}).get("disabled_slots", []))})
        return {"agents": out}

    @route("POST", r"/api/v1/agents/([^/]+)/slots/(\d+)/(enable|disable)")
    def slot_enable(q, b, agent_id, slot, what):
        """``det slot enable|disable`` (reference ``api_agents.go`` EnableSlot / DisableSlot): a
        disabled slot gets no new allocations; one running on it keeps it until it ends."""
        m.iam.require("admin_cluster")
        with m.lock:
            if agent_id not in m.agents:
                raise HTTPError(404, f"agent {agent_id} not found")
            if not m.sched.set_slot_enabled(agent_id, int(slot), what == "enable"):
                raise HTTPError(404, f"slot {slot} of agent {agent_id} not found")
            dis = set(m.agents[agent_id].get("disabled_slots") or [])
            (dis.discard if what == "enable" else dis.add)(int(slot))
            m.agents[agent_id]["disabled_slots"] = sorted(dis)
            m._schedule()
        return {"agent_id": agent_id, "slot_id": int(slot), "enabled": what == "enable"}

    @route("POST", r"/api/v1/agents/([^/]+)/(enable|disable)")
    def agent_enable(q, b, agent_id, what):
        m.iam.require("admin_cluster")
        with m.lock:
            if agent_id in m.agents:
                m.agents[agent_id]["enabled"] = what == "enable"
                m.sched.set_agent_enabled(agent_id, what == "enable")
        return {}

    def _ws_names(ids):
        rows = {int(r["id"]): r["name"] for r in m.db.all("SELECT id, name FROM workspaces")}
        return [rows.get(i, str(i)) for i in ids]

    @route("GET", "/api/v1/resource-pools")
    def pools(q, b):
        with m.lock:
            rows = m.sched.summary()
            for r in rows:
                r["bound_workspaces"] = _ws_names(m.pool_bindings(r["name"]))
        return {"resource_pools": rows}

    def _ws_ids(b):
        ids = [int(w) for w in b.get("workspace_ids") or []]
        for name in b.get("workspace_names") or []:
            ids.append(int(m.iam.workspace(name)["id"]))
        return ids

    @route("GET", r"/api/v1/resource-pools/([^/]+)/workspace-bindings")
    def pool_bindings(q, b, pool):
        if pool not in m.sched.pools:
            raise HTTPError(404, f"resource pool {pool} not found")
        ids = m.pool_bindings(pool)
        return {"workspace_ids": ids, "workspaces": _ws_names(ids)}

    def _bind(mode):
        def fn(q, b, pool):
            m.iam.require("admin_cluster")
            ids = m.set_pool_bindings(pool, _ws_ids(b), mode)
            return {"workspace_ids": ids, "workspaces": _ws_names(ids)}
        return fn

    route("POST", r"/api/v1/resource-pools/([^/]+)/workspace-bindings")(_bind("add"))
    route("PUT", r"/api/v1/resource-pools/([^/]+)/workspace-bindings")(_bind("replace"))
    route("DELETE", r"/api/v1/resource-pools/([^/]+)/workspace-bindings")(_bind("remove"))

    @route("GET", r"/api/v1/workspaces/([^/]+)/available-resource-pools")
    def ws_pools(q, b, ref):
        w = m.iam.workspace(ref)
        m.iam.require("view", w["id"])
        return {"resource_pools": m.pools_for_workspace(int(w["id"]))}

    @route("GET", "/api/v1/resources/allocation/raw")
    def alloc_raw(q, b):
        return {"allocations": m.allocation_usage(_ts(q.get("timestamp_after"), 0.0),
                                                  _ts(q.get("timestamp_before"), time.time() + 1))}

    @route("GET", "/api/v1/resources/allocation/aggregated")
    def alloc_agg(q, b):
        """Slot-hours per day (or month) in [start_date, end_date], by experiment owner, experiment,
        resource pool and task kind (reference ``api_resources.go`` ResourceAllocationAggregated)."""
        import datetime

        period = (q.get("period") or "DAILY").upper()
        d0 = datetime.date.fromisoformat(q["start_date"])
        d1 = datetime.date.fromisoformat(q["end_date"])
        out = []
        day = d0
        while day <= d1:
            if period == "MONTHLY":
                nxt = (day.replace(day=1) + datetime.timedelta(days=32)).replace(day=1)
            else:
                nxt = day + datetime.timedelta(days=1)
            t0 = datetime.datetime.combine(day, datetime.time()).timestamp()
            t1 = datetime.datetime.combine(nxt, datetime.time()).timestamp()
            agg = {"period_start": day.isoformat(), "period": period, "seconds": 0.0, "by_username": {},
                   "by_experiment_id": {}, "by_resource_pool": {}, "by_kind": {}}
            for r in m.allocation_usage(t0, t1):
                ss = r["slot_seconds"]
                agg["seconds"] += ss
                for key, val in (("by_username", r["owner"]), ("by_experiment_id", r["experiment_id"]),
                                 ("by_resource_pool", r["resource_pool"]), ("by_kind", r["kind"])):
                    if val is not None:
                        agg[key][str(val)] = agg[key].get(str(val), 0.0) + ss
            out.append(agg)
            day = nxt
        return {"resource_entries": out}

    @route("GET", "/api/v1/job-queues")
    def jobs(q, b):
        return {"jobs": list(m.sched.requests(q.get("resource_pool") or None).values())}

    # ---------------------------------------------------------------- model registry
    @route("POST", "/api/v1/models")
    def create_model(q, b):
        try:
            mid = m.db.insert("models", name=b["name"], description=b.get("description", ""),
                              metadata=b.get("metadata", {}), labels=b.get("labels", []), creation_time=time.time())
        except Exception as e:
            raise HTTPError(400, f"cannot create model: {e}")
        return {"model": m.db.one("SELECT * FROM models WHERE id=?", [mid])}

    @route("GET", "/api/v1/models")
    def list_models(q, b):
        return {"models": m.db.all("SELECT * FROM models ORDER BY id")}

    @route("GET", r"/api/v1/models/([^/]+)")
    def get_model(q, b, name):
        name = urllib.parse.unquote(name)
        row = m.db.one("SELECT * FROM models WHERE name=?", [name])
        if row is None:
            raise HTTPError(404, f"model {name} not found")
        return {"model": row}

    @route("PATCH", r"/api/v1/models/([^/]+)")
    def patch_model(q, b, name):
        cols = {k: v for k, v in b.items() if k in ("description", "metadata", "labels", "notes", "archived",
                                                    "workspace")}
        if "workspace" in cols:
            m.iam.workspace(cols["workspace"])  # must exist
        m.db.update("models", "name", urllib.parse.unquote(name), **cols)
        return {}

    @route("DELETE", r"/api/v1/models/([^/]+)")
    def del_model(q, b, name):
        row = m.db.one("SELECT id FROM models WHERE name=?", [urllib.parse.unquote(name)])
        if row:
            m.db.execute("DELETE FROM model_versions WHERE model_id=?", [row["id"]])
            m.db.execute("DELETE FROM models WHERE id=?", [row["id"]])
        return {}

    @route("POST", r"/api/v1/models/([^/]+)/versions")
    def register_version(q, b, name):
        name = urllib.parse.unquote(name)
        row = m.db.one("SELECT id FROM models WHERE name=?", [name])
        if row is None:
            raise HTTPError(404, f"model {name} not found")
        if m.db.one("SELECT uuid FROM checkpoints WHERE uuid=?", [b["checkpoint_uuid"]]) is None:
            raise HTTPError(404, f"checkpoint {b['checkpoint_uuid']} not found")
        last = m.db.one("SELECT MAX(version) AS v FROM model_versions WHERE model_id=?", [row["id"]])
        ver = (last["v"] or 0) + 1
        m.db.insert("model_versions", model_id=row["id"], version=ver, checkpoint_uuid=b["checkpoint_uuid"],
                    name=b.get("name") or f"V{ver}", comment=b.get("comment", ""), metadata=b.get("metadata", {}),
                    creation_time=time.time())
        return {"model_version": m.db.one("SELECT * FROM model_versions WHERE model_id=? AND version=?",
                                          [row["id"], ver])}

    @route("GET", r"/api/v1/models/([^/]+)/versions")
    def list_versions(q, b, name):
        row = m.db.one("SELECT id FROM models WHERE name=?", [urllib.parse.unquote(name)])
        if row is None:
            raise HTTPError(404, "model not found")
        return {"model_versions": m.db.all("SELECT * FROM model_versions WHERE model_id=? ORDER BY version",
                                           [row["id"]])}

    def _version_row(name: str, ver: str) -> Dict[str, Any]:
        mrow = m.db.one("SELECT id FROM models WHERE name=?", [urllib.parse.unquote(name)])
        row = m.db.one("SELECT * FROM model_versions WHERE model_id=? AND version=?", [mrow["id"], int(ver)]) \
            if mrow else None
        if row is None:
            raise HTTPError(404, f"model version {name}/{ver} not found")
        return row

    @route("PATCH", r"/api/v1/models/([^/]+)/versions/(\d+)")
    def patch_version(q, b, name, ver):
        row = _version_row(name, ver)
        cols = {k: v for k, v in b.items() if k in ("name", "comment", "metadata", "notes")}
        if "notes" in cols:
            cols["comment"] = cols.pop("notes")
        m.db.update("model_versions", "id", row["id"], **cols)
        return {}

    @route("DELETE", r"/api/v1/models/([^/]+)/versions/(\d+)")
    def del_version(q, b, name, ver):
        row = _version_row(name, ver)
        m.db.execute("DELETE FROM model_versions WHERE id=?", [row["id"]])
        return {}

    # ---------------------------------------------------------------- webhooks / templates
    @route("POST", "/api/v1/webhooks")
    def create_hook(q, b):
        wid = m.db.insert("webhooks", url=b["url"], triggers=b.get("triggers", []),
                          webhook_type=b.get("webhook_type", "DEFAULT"))
        return {"webhook": m.db.one("SELECT * FROM webhooks WHERE id=?", [wid])}

    @route("GET", "/api/v1/webhooks")
    def list_hooks(q, b):
        return {"webhooks": m.db.all("SELECT * FROM webhooks")}

    @route("DELETE", r"/api/v1/webhooks/(\d+)")
    def del_hook(q, b, wid):
        m.db.execute("DELETE FROM webhooks WHERE id=?", [int(wid)])
        return {}

    @route("PUT", r"/api/v1/templates/([^/]+)")
    def put_template(q, b, name):
        m.db.execute("INSERT OR REPLACE INTO templates (name, config) VALUES (?,?)", [name, json.dumps(b["config"])])
        return {}

    @route("GET", "/api/v1/templates")
    def list_templates(q, b):
        return {"templates": m.db.all("SELECT * FROM templates")}

    @route("GET", r"/api/v1/templates/([^/]+)")
    def get_template(q, b, name):
        row = m.db.one("SELECT * FROM templates WHERE name=?", [name])
        if row is None:
            raise HTTPError(404, f"template {name} not found")
        cfg = row["config"]
        return {"template": {"name": row["name"], "config": json.loads(cfg) if isinstance(cfg, str) else cfg}}

    @route("GET", "/metrics")
    def prom(q, b):
        exps = m.db.all("SELECT state, COUNT(*) AS n FROM experiments GROUP BY state")
        lines = ["# TYPE det_slots_total gauge", f"det_slots_total {m.sched.total_slots}",
                 "# TYPE det_slots_used gauge", f"det_slots_used {m.sched.used_slots}",
                 "# TYPE det_experiments gauge"]
        lines += [f'det_experiments{{state="{r["state"]}"}} {r["n"]}' for r in exps]
        return _Raw("\n".join(lines) + "\n", "text/plain; version=0.0.4")

    add_webui_routes(route, _Raw)
    return routes


_LOOPBACK = frozenset(("127.0.0.1", "localhost", "::1"))


def public_task(row: Dict[str, Any]) -> Dict[str, Any]:
    """A task row as the API shows it: a shell server's key stays inside the master."""
    px = row.get("proxy")
    if isinstance(px, dict) and "shell_key" in px:
        row = dict(row, proxy={k: v for k, v in px.items() if k != "shell_key"})
    return row


def _may_use_proxy(iam: Any, task_cfg: Dict[str, Any]) -> bool:
    """Reference ``processProxyAuthentication`` (CanGetNSC / CanGetTensorboard): the owner and admins
    always; in rbac mode also users with view permission on the task's workspace."""
    if iam is None or iam.mode == "none":
        return True
    u = iam.current()
    if u["admin"] or (task_cfg.get("owner_id") is not None and task_cfg.get("owner_id") == u["id"]):
        return True
    return iam.mode == "rbac" and iam.can("view", task_cfg.get("workspace_id"), None, user=u) and \
        task_cfg.get("workspace_id") is not None


def _strip_auth_cookie(cookie: str) -> str:
    """The master's own session cookie never reaches the proxied service."""
    kept = [c.strip() for c in cookie.split(";") if c.strip() and c.strip().partition("=")[0] != "auth"]
    return "; ".join(kept)


class _Raw:
    def __init__(self, body: Any, ctype: str) -> None:  # str or bytes
        self.body = body
        self.ctype = ctype


class _Handler(BaseHTTPRequestHandler):
    routes: List[Route] = []
    master: Optional[Master] = None
    protocol_version = "HTTP/1.1"

    def log_message(self, fmt: str, *args: Any) -> None:
        logger.debug("%s - " + fmt, self.address_string(), *args)

    def _proxy(self, method: str, parsed: Any, raw: bytes) -> None:
        """``/proxy/<task_id>/<path>``: forward the request to the task's registered service
        (notebook / TensorBoard / any NTSC that posted ``/api/v1/tasks/<id>/proxy``), as the
        reference master's task proxy (``master/internal/proxy``) -- plain HTTP, no websockets."""
        import http.client

        parts = parsed.path.split("/", 3)  # ['', 'proxy', task_id, rest]
        task_id = parts[2] if len(parts) > 2 else ""
        rest = "/" + (parts[3] if len(parts) > 3 else "")
        iam = self.master.iam if self.master else None
        try:
            if iam is not None:
                auth = self.headers.get("Authorization")
                if auth is None:  # browsers: the session token as a cookie
                    for c in (self.headers.get("Cookie") or "").split(";"):
                        k, _, v = c.strip().partition("=")
                        if k == "auth":
                            auth = f"Bearer {v}"
                iam.set_current(iam.authenticate(auth))
            row = self.master.db.one("SELECT proxy, config FROM tasks WHERE id=?", [task_id]) if self.master else None
            if row is None or not _may_use_proxy(iam, row.get("config") or {}):
                raise HTTPError(404, f"task {task_id} not found")  # no existence leak to other users
            px = row.get("proxy")
            if not px or not px.get("port"):
                raise HTTPError(404, f"task {task_id} has no proxied service (yet)")
            if rest == "/_tunnel":
                self._tunnel(px)
                return
            if px.get("tunnel"):
                raise HTTPError(400, f"task {task_id} serves a shell: connect with `det shell open {task_id}`")
            conn = http.client.HTTPConnection(px.get("host") or "127.0.0.1", int(px["port"]), timeout=60)
            hdrs = {k: v for k, v in self.headers.items() if k.lower() not in ("host", "authorization", "content-length",
                                                                             "connection", "cookie")}
            cookie = _strip_auth_cookie(self.headers.get("Cookie") or "")
            if cookie:
                hdrs["Cookie"] = cookie
            conn.request(method, rest + (f"?{parsed.query}" if parsed.query else ""), body=raw or None, headers=hdrs)
            resp = conn.getresponse()
            data = resp.read()
            self.send_response(resp.status)
            for k, v in resp.getheaders():
                if k.lower() not in ("transfer-encoding", "connection", "content-length"):
                    self.send_header(k, v)
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)
            conn.close()
        except (HTTPError, AuthError) as e:
            data = json.dumps({"error": e.message}).encode()
            self.send_response(e.status)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)
        except OSError as e:
            data = json.dumps({"error": f"proxied service unreachable: {e}"}).encode()
            self.send_response(502)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

    def _tunnel(self, px: Dict[str, Any]) -> None:
        """``/proxy/<task>/_tunnel`` with ``Upgrade: damd-tunnel``: a raw byte stream to the task's
        shell server (exec/shell.py).  The user is already authorised for the task (``_proxy``); the
        master sends the task's shell key as the first line, answers 101 and relays both ways until
        either side closes (reference: the master's TCP proxy behind ``det shell``'s ssh tunnel)."""
        import select
        import socket

        if (self.headers.get("Upgrade") or "").lower() != "damd-tunnel" or not px.get("tunnel"):
            raise HTTPError(400, "this endpoint needs 'Upgrade: damd-tunnel' on a shell task")
        up = socket.create_connection((px.get("host") or "127.0.0.1", int(px["port"])), timeout=10)
        up.settimeout(None)
        up.sendall(b"DAMD-SHELL " + str(px.get("shell_key") or "").encode() + b"\n")
        self.send_response(101)
        self.send_header("Upgrade", "damd-tunnel")
        self.send_header("Connection", "Upgrade")
        self.end_headers()
        self.wfile.flush()
        self.close_connection = True
        down = self.connection
        try:
            while True:
                r, _, _ = select.select([down, up], [], [], 60)
                if not r:
                    continue
                for src, dst in ((down, up), (up, down)):
                    if src in r:
                        data = src.recv(65536)
                        if not data:
                            return
                        dst.sendall(data)
        except OSError:
            return
        finally:
            up.close()

    def _dispatch(self, method: str) -> None:
        parsed = urllib.parse.urlparse(self.path)
        q = {k: v[-1] for k, v in urllib.parse.parse_qs(parsed.query).items()}
        n = int(self.headers.get("Content-Length") or 0)
        raw = self.rfile.read(n) if n else b""
        if parsed.path.startswith("/proxy/"):
            self._proxy(method, parsed, raw)
            return
        status, ctype = 200, "application/json"
        try:
            iam = self.master.iam if self.master else None
            if iam is not None:
                iam.set_current(None)
                if parsed.path.startswith("/api/") and parsed.path != "/api/v1/auth/login":
                    try:
                        iam.set_current(iam.authenticate(self.headers.get("Authorization")))
                    except AuthError as e:
                        raise HTTPError(e.status, e.message)
            body = json.loads(raw) if raw else {}
            for meth, pat, fn in self.routes:
                if meth != method:
                    continue
                mm = pat.match(parsed.path)
                if mm:
                    out = fn(q, body, *mm.groups())
                    break
            else:
                raise HTTPError(404, f"no route {method} {parsed.path}")
            if isinstance(out, _Raw):
                data, ctype = (out.body if isinstance(out.body, bytes) else out.body.encode()), out.ctype
            else:
                data = json.dumps(out, default=str).encode()
        except (HTTPError, AuthError) as e:
            status, data = e.status, json.dumps({"error": e.message}).encode()
        except ValueError as e:  # invalid request content (e.g. an unknown resource pool)
            status, data = 400, json.dumps({"error": str(e)}).encode()
        except KeyError as e:
            status, data = 404, json.dumps({"error": str(e)}).encode()
        except Exception as e:  # noqa: BLE001
            logger.exception("request failed")
            status, data = 500, json.dumps({"error": repr(e)}).encode()
        self.send_response(status)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def do_GET(self) -> None:
        self._dispatch("GET")

    def do_POST(self) -> None:
        self._dispatch("POST")

    def do_DELETE(self) -> None:
        self._dispatch("DELETE")

    def do_PATCH(self) -> None:
        self._dispatch("PATCH")

    def do_PUT(self) -> None:
        self._dispatch("PUT")


class MasterServer:
    def __init__(self, master: Master, host: str = "127.0.0.1", port: int = 8080) -> None:
        handler = type("Handler", (_Handler,), {"routes": build_routes(master), "master": master})
        self.httpd = ThreadingHTTPServer((host, port), handler)
        self.httpd.daemon_threads = True
        self.master = master
        self.port = self.httpd.server_address[1]
        self.thread: Optional[threading.Thread] = None

    def start(self) -> "MasterServer":
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True, name="master-http")
        self.thread.start()
        return self

    def serve_forever(self) -> None:
        self.httpd.serve_forever()

    def stop(self) -> None:
        self.master.close()
        self.httpd.shutdown()
        self.httpd.server_close()
