"""Experiment / trial / model / job / task / template management verbs end to end on a CPU
cluster (in-process master + agent running real trials), plus ``resources.max_slots``
enforcement (reference: ``e2e_tests/tests/cluster/test_experiment_*``, ``test_checkpoints.py``)."""

import contextlib
import io
import os
import tarfile
import time

import pytest

from tests.test_e2e_cpu import HP, _create, _trials, _wait, cluster  # noqa: F401  (fixture)


def det(cluster, *args):
    from determined_amd.cli import main

    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        rc = main(["-m", cluster["url"], *args])
    assert rc in (0, None), out.getvalue()
    return out.getvalue()


def test_experiment_management_verbs(cluster, tmp_path, monkeypatch):  # noqa: F811
    monkeypatch.chdir(tmp_path)
    eid = _create(cluster, {"name": "mgmt", "hyperparameters": HP,
                            "searcher": {"name": "single", "metric": "validation_loss",
                                         "max_length": {"batches": 6}}, "min_validation_period": {"batches": 3}})
    assert _wait(cluster, eid)["state"] == "COMPLETED"
    s = cluster["session"]
    assert "name: mgmt" in det(cluster, "experiment", "config", str(eid))
    out = det(cluster, "experiment", "download-model-def", str(eid)).strip()
    with tarfile.open(out) as tf:
        assert any(n.endswith("model_def.py") for n in tf.getnames())
    det(cluster, "experiment", "label", "add", str(eid), "baseline")
    assert s.get(f"/api/v1/experiments/{eid}")["experiment"]["labels"] == ["baseline"]
    det(cluster, "experiment", "label", "remove", str(eid), "baseline")
    det(cluster, "experiment", "set", "description", str(eid), "tuned")
    det(cluster, "experiment", "set", "priority", str(eid), "10")
    det(cluster, "experiment", "set", "weight", str(eid), "2.5")
    det(cluster, "experiment", "set", "max-slots", str(eid), "1")
    det(cluster, "experiment", "set", "log-retention", str(eid), "--days", "7")
    cfg = s.get(f"/api/v1/experiments/{eid}")["config"]
    assert cfg["resources"]["priority"] == 10 and cfg["resources"]["weight"] == 2.5
    assert cfg["resources"]["max_slots"] == 1 and cfg["retention_policy"]["log_retention_days"] == 7
    assert s.get(f"/api/v1/experiments/{eid}")["experiment"]["description"] == "tuned"
    det(cluster, "experiment", "set", "gc-policy", str(eid), "--save-trial-latest", "1", "--save-trial-best", "0",
        "--save-experiment-best", "0")
    ck = [c for c in s.get(f"/api/v1/experiments/{eid}/checkpoints")["checkpoints"] if c["state"] == "COMPLETED"]
    assert len(ck) == 1
    out = det(cluster, "experiment", "download", str(eid), "-o", str(tmp_path / "dl")).strip()
    assert os.path.isdir(out) and os.listdir(out)
    det(cluster, "experiment", "delete-tb-files", str(eid))
    # trial verbs
    (t,) = _trials(cluster, eid)
    out = det(cluster, "trial", "download", str(t["id"]), "--latest", "-o", str(tmp_path / "tdl")).strip()
    assert os.path.isdir(out)
    out = det(cluster, "trial", "support-bundle", str(t["id"]), "-o", str(tmp_path)).strip()
    with tarfile.open(out) as tf:
        names = tf.getnames()
    assert any(n.endswith("trial_logs.txt") for n in names) and any(n.endswith("metrics.json") for n in names)
    det(cluster, "trial", "set", "log-retention", str(t["id"]), "--days", "0")
    # continue: new single-trial experiment warm-started from the parent's checkpoint
    out = det(cluster, "experiment", "continue", str(eid), "--config", "searcher.max_length.batches=9")
    new = int(out.strip().split()[-1])
    e2 = _wait(cluster, new)
    assert e2["state"] == "COMPLETED" and e2["parent_id"] == eid
    (t2,) = _trials(cluster, new)
    assert t2["total_batches"] >= 9


def test_model_job_task_template_verbs(cluster, tmp_path):  # noqa: F811
    s = cluster["session"]
    det(cluster, "workspace", "create", "ws-models")
    eid = _create(cluster, {"name": "for-model", "hyperparameters": HP,
                            "searcher": {"name": "single", "metric": "validation_loss", "max_length": {"batches": 2}}})
    assert _wait(cluster, eid)["state"] == "COMPLETED"
    ck = s.get(f"/api/v1/experiments/{eid}/checkpoints")["checkpoints"][0]["uuid"]
    det(cluster, "model", "create", "m-extra")
    det(cluster, "model", "register-version", "m-extra", ck)
    assert ck in det(cluster, "model", "list-versions", "m-extra")
    det(cluster, "model", "move", "m-extra", "ws-models")
    assert s.get("/api/v1/models/m-extra")["model"]["workspace"] == "ws-models"
    det(cluster, "model", "delete", "m-extra")
    with pytest.raises(Exception):
        s.get("/api/v1/models/m-extra")
    # job queue: a paused experiment's priority via update-batch
    eid2 = _create(cluster, {"name": "queued", "hyperparameters": HP,
                             "searcher": {"name": "single", "metric": "validation_loss",
                                          "max_length": {"batches": 2}}}, activate=False)
    det(cluster, "job", "update-batch", f"exp-{eid2}:priority=5", f"exp-{eid2}:weight=3")
    r = s.get(f"/api/v1/experiments/{eid2}")["config"]["resources"]
    assert r["priority"] == 5 and r["weight"] == 3.0
    s.post(f"/api/v1/experiments/{eid2}/kill", {})
    # task verbs
    tid = s.post("/api/v1/commands", {"command": "sleep 30", "slots": 0})["task_id"]
    assert tid in det(cluster, "task", "config", tid)
    det(cluster, "task", "kill", tid)
    # templates
    (tmp_path / "tpl.yaml").write_text("resources:\n  slots_per_trial: 1\n")
    det(cluster, "template", "set", "t1", str(tmp_path / "tpl.yaml"))
    assert "slots_per_trial: 1" in det(cluster, "template", "describe", "t1")
    det(cluster, "template", "remove", "t1")
    with pytest.raises(Exception):
        s.get("/api/v1/templates/t1")


def test_max_slots_limits_concurrent_trials(cluster):  # noqa: F811
    s = cluster["session"]
    eid = _create(cluster, {"name": "capped", "hyperparameters": {"global_batch_size": 16,
                                                                 "lr": {"type": "categorical",
                                                                        "vals": [0.01, 0.02, 0.05]}},
                            "resources": {"slots_per_trial": 1, "max_slots": 1},
                            "searcher": {"name": "grid", "metric": "validation_loss", "max_length": {"batches": 8}}})
    peak = 0
    t0 = time.time()
    while time.time() - t0 < 240:
        allocs = [a for a in s.get("/api/v1/allocations")["allocations"]
                  if a.get("experiment_id") == eid]
        peak = max(peak, len([a for a in allocs if a.get("state") in ("ASSIGNED", "RUNNING")]))
        if s.get(f"/api/v1/experiments/{eid}")["experiment"]["state"] == "COMPLETED":
            break
        time.sleep(0.1)
    assert s.get(f"/api/v1/experiments/{eid}")["experiment"]["state"] == "COMPLETED"
    assert len(_trials(cluster, eid)) == 3 and peak == 1
