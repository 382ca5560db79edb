"""Experiment / trial / template / job-queue management routes behind ``det experiment
config|continue|set ...|label|delete-tb-files``, ``det trial set|support-bundle``, ``det job
update-batch`` and ``det template describe|remove`` (reference: ``master/internal/api_experiment.go``
PatchExperiment / ContinueExperiment / DeleteTensorboardFiles, ``api_trials.go``,
``api_job.go`` UpdateJobQueue, ``api_template.go``)."""

import io
import json
import shutil
import tarfile
import time
from typing import Any, Callable


def add_exp_routes(route: Callable[[str, str], Callable], m: Any) -> None:
    from determined_amd.master._server import HTTPError, _guard_exp

    @route("POST", r"/api/v1/experiments/(\d+)/continue")
    def continue_exp(q, b, eid):
        _guard_exp(m, eid, "edit")
        try:
            new = m.continue_experiment(int(eid), b.get("overrides") or {})
        except ValueError as e:
            raise HTTPError(400, str(e))
        return {"experiment_id": new}

    @route("POST", r"/api/v1/experiments/(\d+)/resources")
    def set_resources(q, b, eid):
        _guard_exp(m, eid, "edit")
        kw = {}
        if "max_slots" in b:
            kw["max_slots"] = b["max_slots"]
        m.set_experiment_resources(int(eid), weight=b.get("weight"), priority=b.get("priority"), **kw)
        return {}

    @route("PATCH", r"/api/v1/experiments/(\d+)/config/([a-z_]+)")
    def patch_cfg(q, b, eid, section):
        _guard_exp(m, eid, "edit")
        try:
            cfg = m.patch_experiment_config(int(eid), section, b)
        except ValueError as e:
            raise HTTPError(400, str(e))
        if section == "checkpoint_storage":  # a new GC policy applies right away
            m.gc_experiment_checkpoints(int(eid))
        return {"config": cfg}

    @route("POST", r"/api/v1/experiments/(\d+)/labels")
    def labels(q, b, eid):
        _guard_exp(m, eid, "edit")
        row = m.db.one("SELECT labels FROM experiments WHERE id=?", [int(eid)])
        cur = list(row["labels"] or [])
        for lab in b.get("add", []):
            if lab not in cur:
                cur.append(lab)
        cur = [x for x in cur if x not in set(b.get("remove", []))]
        m.db.update("experiments", "id", int(eid), labels=cur)
        return {"labels": cur}

    @route("DELETE", r"/api/v1/experiments/(\d+)/tensorboard-files")
    def delete_tb(q, b, eid):
        _guard_exp(m, eid, "edit")
        from determined_amd import storage

        row = m.db.one("SELECT config FROM experiments WHERE id=?", [int(eid)])
        cfg = row["config"]
        sm = storage.build(cfg.get("tensorboard_storage") or cfg["checkpoint_storage"])
        import os

        d = os.path.join(sm._base_path, "tensorboard", "experiment", str(int(eid)))
        existed = os.path.isdir(d)
        shutil.rmtree(d, ignore_errors=True)
        return {"deleted": existed}

    @route("PATCH", r"/api/v1/trials/(\d+)")
    def patch_trial(q, b, tid):
        row = m.db.one("SELECT experiment_id FROM trials WHERE id=?", [int(tid)])
        if row is None:
            raise HTTPError(404, f"trial {tid} not found")
        _guard_exp(m, row["experiment_id"], "edit")
        if "state" in b or b.get("heartbeat"):
            # unmanaged trials report their own state and heartbeats (core/_heartbeat.py)
            try:
                m.unmanaged_trial_report(int(tid), b.get("state"))
            except ValueError as e:
                raise HTTPError(400, str(e))
        if "log_retention_days" in b:
            # per-trial retention: logs of this trial are dropped once it is older than N days
            v = b["log_retention_days"]
            m.db.update("trials", "id", int(tid), log_retention_days=None if v is None else int(v))
        return {}

    @route("GET", r"/api/v1/trials/(\d+)/support-bundle")
    def support_bundle(q, b, tid):
        """tar.gz (base64) of the trial record, its metrics, checkpoints and logs."""
        import base64

        t = m.db.one("SELECT * FROM trials WHERE id=?", [int(tid)])
        if t is None:
            raise HTTPError(404, f"trial {tid} not found")
        e = m.db.one("SELECT id, name, state, config FROM experiments WHERE id=?", [t["experiment_id"]])
        files = {
            "trial.json": json.dumps(t, default=str, indent=2),
            "experiment.json": json.dumps(e, default=str, indent=2),
            "metrics.json": json.dumps(m.db.all("SELECT * FROM metrics WHERE trial_id=? ORDER BY id", [int(tid)]),
                                       default=str),
            "checkpoints.json": json.dumps(m.db.all("SELECT * FROM checkpoints WHERE trial_id=?", [int(tid)]),
                                           default=str),
            "trial_logs.txt": "\n".join(r["log"] for r in m.get_logs(f"trial-{int(tid)}", 0, 1_000_000)),
            "master_info.json": json.dumps({"cluster_id": m.cluster_id, "time": time.time()}),
        }
        buf = io.BytesIO()
        with tarfile.open(fileobj=buf, mode="w:gz") as tf:
            for name, text in files.items():
                data = text.encode()
                ti = tarfile.TarInfo(f"bundle-trial-{int(tid)}/{name}")
                ti.size = len(data)
                ti.mtime = int(time.time())
                tf.addfile(ti, io.BytesIO(data))
        return {"b64_tgz": base64.b64encode(buf.getvalue()).decode()}

    @route("POST", "/api/v1/job-queues/update")
    def update_jobs(q, b):
        for u in b.get("updates", []):
            job = str(u["job_id"])
            if not job.startswith("exp-"):  # a command / notebook / shell / tensorboard task
                if m.db.one("SELECT id FROM tasks WHERE id=?", [job]) is None:
                    raise HTTPError(404, f"job {job} not found")
                m.set_task_priority(job, u.get("priority"), u.get("weight"))
                continue
            eid = int(job.split("-", 1)[1])
            _guard_exp(m, eid, "edit")
            m.set_experiment_resources(eid, weight=u.get("weight"), priority=u.get("priority"))
        return {}

    @route("DELETE", r"/api/v1/templates/([^/]+)")
    def del_template(q, b, name):
        m.db.execute("DELETE FROM templates WHERE name=?", [name])
        return {}

