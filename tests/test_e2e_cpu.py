"""Cluster end to end on CPU: in-process master + agent (2 CPU slots) running real trial
processes (``exec.harness`` under the agent).  Covers experiment lifecycle, searchers,
restarts, InvalidHP, checkpoints/GC, logs, model registry and the ``det`` CLI."""

import base64
import contextlib
import io
import json
import os
import pathlib
import tempfile
import threading
import time

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
TINY = ROOT / "tests" / "fixtures" / "tiny_trial"


@pytest.fixture(scope="module")
def cluster():
    from determined_amd.agent import Agent
    from determined_amd.common.api import Session
    from determined_amd.master import start_master

    srv = start_master()
    url = f"http://127.0.0.1:{srv.port}"
    work = tempfile.mkdtemp()
    ag = Agent(url, "e2e-agent", slots=2, work_root=work)
    th = threading.Thread(target=ag.run, daemon=True)
    th.start()
    ck = tempfile.mkdtemp()
    yield {"url": url, "session": Session(url), "ckpt": ck, "master": srv}
    if hasattr(ag, "stop"):
        ag.stop()
    srv.stop() if hasattr(srv, "stop") else None


def _create(cl, cfg, model_dir=TINY, activate=True):
    from determined_amd.cli import tar_model_dir

    cfg = dict(cfg)
    cfg.setdefault("checkpoint_storage", {"type": "shared_fs", "host_path": cl["ckpt"]})
    cfg.setdefault("entrypoint", "model_def:TinyTrial")
    r = cl["session"].post("/api/v1/experiments", {"config": cfg, "activate": activate,
                                                   "model_def": base64.b64encode(tar_model_dir(str(model_dir))).decode()})
    return r["experiment"]["id"]


def _wait(cl, eid, states=("COMPLETED", "ERROR", "CANCELED"), timeout=240):
    t0 = time.time()
    while time.time() - t0 < timeout:
        e = cl["session"].get(f"/api/v1/experiments/{eid}")["experiment"]
        if e["state"] in states:
            return e
        time.sleep(0.5)
    raise TimeoutError(f"experiment {eid} stuck in {e['state']}")


def _trials(cl, eid):
    return cl["session"].get(f"/api/v1/experiments/{eid}/trials")["trials"]


HP = {"lr": 0.1, "global_batch_size": 16}


def test_single_trial(cluster):
    eid = _create(cluster, {"name": "single", "hyperparameters": HP,
                            "searcher": {"name": "single", "metric": "validation_loss", "max_length": {"batches": 12}},
                            "min_validation_period": {"batches": 6}})
    e = _wait(cluster, eid)
    assert e["state"] == "COMPLETED"
    (t,) = _trials(cluster, eid)
    assert t["state"] == "COMPLETED" and t["total_batches"] == 12
    s = cluster["session"]
    ms = s.get(f"/api/v1/trials/{t['id']}/metrics")
    text = json.dumps(ms)
    assert "validation_loss" in text and "loss" in text
    cks = s.get(f"/api/v1/experiments/{eid}/checkpoints")["checkpoints"]
    assert cks and all(os.path.isdir(os.path.join(cluster["ckpt"], c["uuid"])) for c in cks)
    logs = s.get(f"/api/v1/tasks/trial-{t['id']}/logs")["logs"]
    assert any("rank" in l["log"] or "INFO" in l["log"] for l in logs)


def test_adaptive_asha(cluster):
    eid = _create(cluster, {
        "name": "asha",
        "hyperparameters": {"global_batch_size": 16, "lr": {"type": "log", "minval": -3, "maxval": 0, "base": 10}},
        "searcher": {"name": "adaptive_asha", "metric": "validation_loss", "max_length": {"batches": 16},
                     "max_trials": 4, "max_rungs": 2, "divisor": 4, "mode": "aggressive", "max_concurrent_trials": 2}})
    e = _wait(cluster, eid)
    assert e["state"] == "COMPLETED"
    ts = _trials(cluster, eid)
    assert len(ts) == 4 and all(t["state"] == "COMPLETED" for t in ts)
    lengths = sorted(t["total_batches"] for t in ts)
    assert lengths[-1] == 16 and lengths[0] < 16  # promoted vs stopped at the lower rung


def test_restart_and_invalid_hp(cluster):
    marker = os.path.join(tempfile.mkdtemp(), "crashed")
    eid = _create(cluster, {"name": "flaky", "max_restarts": 2,
                            "hyperparameters": {**HP, "crash_marker": marker},
                            "searcher": {"name": "single", "metric": "validation_loss", "max_length": {"batches": 6}}})
    e = _wait(cluster, eid)
    (t,) = _trials(cluster, eid)
    assert e["state"] == "COMPLETED" and t["restarts"] == 1 and os.path.exists(marker)
    eid2 = _create(cluster, {"name": "invalid", "hyperparameters": {**HP, "invalid": True},
                             "searcher": {"name": "single", "metric": "validation_loss",
                                          "max_length": {"batches": 6}}})
    e2 = _wait(cluster, eid2)
    (t2,) = _trials(cluster, eid2)
    assert e2["state"] == "COMPLETED" and t2["restarts"] == 0 and t2["total_batches"] == 0


def test_pause_activate_and_kill(cluster):
    s = cluster["session"]
    eid = _create(cluster, {"name": "paused", "hyperparameters": HP,
                            "searcher": {"name": "single", "metric": "validation_loss", "max_length": {"batches": 6}}},
                  activate=False)
    time.sleep(1.5)
    assert s.get(f"/api/v1/experiments/{eid}")["experiment"]["state"] == "PAUSED"
    assert _trials(cluster, eid)[0]["total_batches"] == 0
    s.post(f"/api/v1/experiments/{eid}/activate", {})
    assert _wait(cluster, eid)["state"] == "COMPLETED"
    eid2 = _create(cluster, {"name": "killed", "hyperparameters": HP,
                             "searcher": {"name": "single", "metric": "validation_loss",
                                          "max_length": {"batches": 100000}}})
    time.sleep(2)
    s.post(f"/api/v1/experiments/{eid2}/kill", {})
    assert _wait(cluster, eid2)["state"] == "CANCELED"


def test_grid_and_model_registry_and_cli(cluster):
    from determined_amd.cli import main as det

    eid = _create(cluster, {"name": "grid",
                            "hyperparameters": {"global_batch_size": 16,
                                                "lr": {"type": "categorical", "vals": [0.01, 0.1]}},
                            "searcher": {"name": "grid", "metric": "validation_loss", "max_length": {"batches": 4}}})
    assert _wait(cluster, eid)["state"] == "COMPLETED"
    ts = _trials(cluster, eid)
    assert sorted(t["hparams"]["lr"] for t in ts) == [0.01, 0.1]
    s = cluster["session"]
    ck = s.get(f"/api/v1/experiments/{eid}/checkpoints")["checkpoints"][0]["uuid"]
    s.post("/api/v1/models", {"name": "tiny-model", "description": "e2e"})
    s.post("/api/v1/models/tiny-model/versions", {"checkpoint_uuid": ck})
    vs = s.get("/api/v1/models/tiny-model/versions")
    assert json.dumps(vs).count(ck) >= 1
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        rc = det(["-m", cluster["url"], "experiment", "list"])
    assert rc in (0, None) and "grid" in out.getvalue()
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        det(["-m", cluster["url"], "agent", "list"])
    assert "e2e-agent" in out.getvalue()


def test_sdk_client(cluster):
    from determined_amd.experimental import client

    client.login(cluster["url"])
    exp = client.create_experiment(
        {"name": "sdk", "hyperparameters": HP, "entrypoint": "model_def:TinyTrial",
         "checkpoint_storage": {"type": "shared_fs", "host_path": cluster["ckpt"]},
         "searcher": {"name": "single", "metric": "validation_loss", "max_length": {"batches": 8}},
         "min_validation_period": {"batches": 4}}, str(TINY))
    assert exp.wait(interval=0.5, timeout=180) == client.ExperimentState.COMPLETED
    exp.add_label("fast")
    exp.set_description("sdk test")
    exp.reload()
    assert "fast" in exp.labels
    (trial,) = exp.list_trials()
    assert trial.state == client.TrialState.COMPLETED
    assert list(trial.stream_validation_metrics())
    assert any(trial.logs())
    best = exp.top_checkpoint()
    assert best.steps_completed in (4, 8)
    with tempfile.TemporaryDirectory() as d:
        p = best.download(os.path.join(d, "ck"))
        assert os.path.exists(os.path.join(p, "state_dict.pth"))
        code = exp.download_code(os.path.join(d, "code"))
        assert os.path.exists(os.path.join(code, "model_def.py"))
    best.add_metadata({"note": "best"})
    assert client.get_checkpoint(best.uuid).metadata["note"] == "best"
    model = client.create_model("sdk-model", labels=["x"])
    v = model.register_version(best.uuid)
    v.set_notes("first")
    assert model.get_version().model_version == 1 and model.get_version().notes == "first"
    assert [m.name for m in client.list_models(labels=["x"])] == ["sdk-model"]
    v.delete()
    assert model.get_version() is None


def test_core_v2_unmanaged(cluster):
    from determined_amd.experimental import client, core_v2

    defaults = core_v2.DefaultConfig(name="unmanaged-run", hparams={"lr": 0.5},
                                     checkpoint_storage={"type": "shared_fs", "host_path": cluster["ckpt"]})
    um = core_v2.UnmanagedConfig(external_experiment_id="ext-exp-1", external_trial_id="ext-trial-1")
    core_v2.init(defaults=defaults, unmanaged=um, master=cluster["url"])
    tid = core_v2.info.trial.trial_id
    eid = core_v2.info.trial.experiment_id
    for step in (1, 2, 3):
        core_v2.train.report_training_metrics(steps_completed=step, metrics={"loss": 1.0 / step})
    core_v2.train.report_validation_metrics(steps_completed=3, metrics={"unmanaged": 0.25})
    with core_v2.checkpoint.store_path({"steps_completed": 3}) as (path, uuid):
        (path / "w.txt").write_text("weights")
    core_v2.close()
    client.login(cluster["url"])
    exp = client.get_experiment(eid)
    assert exp.state == client.ExperimentState.COMPLETED
    (t,) = exp.list_trials()
    assert t.id == tid and t.hparams == {"lr": 0.5}
    assert len(list(t.stream_training_metrics())) == 3
    assert [c.uuid for c in t.list_checkpoints()] == [uuid]
    # resuming with the same external ids reuses the experiment and trial
    core_v2.init(defaults=defaults, unmanaged=um, master=cluster["url"])
    assert core_v2.info.trial.trial_id == tid and core_v2.info.latest_checkpoint == uuid
    core_v2.close()


def test_custom_searcher_local_runner(cluster):
    import uuid as uuidlib

    from determined_amd import searcher as det_searcher

    class TwoTrials(det_searcher.SearchMethod):
        def __init__(self):
            self.created = 0

        def initial_operations(self, st):
            ops = []
            for lr in (0.05, 0.2):
                rid = uuidlib.uuid4()
                ops += [det_searcher.Create(rid, {"lr": lr, "global_batch_size": 16}, checkpoint=None),
                        det_searcher.ValidateAfter(rid, 4)]
            return ops

        def on_trial_created(self, st, rid):
            self.created += 1
            return []

        def on_validation_completed(self, st, rid, metric, length):
            if length < 8:
                return [det_searcher.ValidateAfter(rid, 8)]
            return [det_searcher.Close(rid)]

        def on_trial_closed(self, st, rid):
            if len(st.trials_closed) == 2:
                return [det_searcher.Shutdown()]
            return []

        def progress(self, st):
            return len(st.trials_closed) / 2

        def on_trial_exited_early(self, st, rid, reason):
            return [det_searcher.Shutdown(failure=True)]

    from determined_amd.common.api import Session

    with tempfile.TemporaryDirectory() as d:
        method = TwoTrials()
        runner = det_searcher.LocalSearchRunner(method, pathlib.Path(d), session=Session(cluster["url"]))
        cfg = {"name": "custom", "entrypoint": "model_def:TinyTrial",
               "checkpoint_storage": {"type": "shared_fs", "host_path": cluster["ckpt"]},
               "searcher": {"name": "custom", "metric": "validation_loss"}, "hyperparameters": HP}
        eid = runner.run(cfg, model_dir=str(TINY))
        assert (pathlib.Path(d) / "searcher_state.json").exists()
    e = _wait(cluster, eid)
    assert e["state"] == "COMPLETED" and method.created == 2
    ts = _trials(cluster, eid)
    assert sorted(t["total_batches"] for t in ts) == [8, 8]


def test_log_policy_cancel_retries_and_retention(cluster):
    eid = _create(cluster, {"name": "logpolicy", "max_restarts": 5, "hyperparameters": HP,
                            "entrypoint": "model_def:NoisyFailTrial",
                            "log_policies": [{"pattern": "ECC error", "action": {"type": "cancel_retries"}},
                                             {"pattern": "ECC error", "action": {"type": "exclude_node"}}],
                            "retention_policy": {"log_retention_days": 0},
                            "searcher": {"name": "single", "metric": "validation_loss",
                                         "max_length": {"batches": 6}}})
    e = _wait(cluster, eid)
    (t,) = _trials(cluster, eid)
    assert e["state"] == "ERROR" and t["state"] == "ERROR" and t["restarts"] == 1  # no further retries
    m = cluster["master"].master
    (tr,) = m.experiments[eid].trials.values()
    assert tr.no_retry and tr.excluded_agents == ["e2e-agent"]
    assert m.cleanup_logs(now=time.time() + 10) > 0


def test_scheduler_excluded_agents():
    from determined_amd._native import load

    n = load()
    s = n.Scheduler(n.Policy.PRIORITY, n.Fit.BEST, True)
    s.add_agent("a", 2)
    s.add_agent("b", 2)
    s.add_request("r1", "j1", 2, excluded_agents=["a"])
    d = s.schedule()
    assert d["allocated"] == ["r1"]
    assert [ag for ag, _ in s.requests()["r1"]["assignment"]] == ["b"]
    s.add_request("r2", "j2", 2, excluded_agents=["a"])
    assert s.schedule()["allocated"] == []  # only "a" is free and it is excluded


def test_trial_source_info_links_inference_metrics():
    """``core_context.experimental.report_task_using_checkpoint / _model_version`` (reference
    core/_experimental.py + api_trials.go ReportTrialSourceInfo): metrics an inference task
    reports become the checkpoint's / model version's ``get_metrics()``."""
    import uuid as _uuid

    from determined_amd.common.api import Session
    from determined_amd.core import ExperimentalCoreContext
    from determined_amd.experimental import client
    from determined_amd.master import start_master

    srv = start_master()
    try:
        url = f"http://127.0.0.1:{srv.port}"
        s = Session(url)
        cfg = {"name": "src", "hyperparameters": {}, "searcher": {"name": "single", "metric": "loss",
                                                                 "max_length": {"batches": 1}}}
        eid = s.post("/api/v1/unmanaged/experiments", {"config": cfg})["experiment"]["id"]
        train_tid = s.post(f"/api/v1/unmanaged/experiments/{eid}/trials", {"hparams": {}})["trial_id"]
        infer_tid = s.post(f"/api/v1/unmanaged/experiments/{eid}/trials", {"hparams": {}})["trial_id"]
        ck = str(_uuid.uuid4())
        s.post("/api/v1/checkpoints", {"uuid": ck, "trial_id": train_tid, "steps_completed": 1,
                                       "resources": {}, "metadata": {}})
        s.post(f"/api/v1/trials/{train_tid}/metrics", {"group": "validation", "steps_completed": 1,
                                                       "metrics": {"loss": 9.0}})
        s.post(f"/api/v1/trials/{infer_tid}/metrics", {"group": "inference", "steps_completed": 5,
                                                       "metrics": {"accuracy": 0.75}})
        client.login(url)
        ckpt = client.get_checkpoint(ck)
        assert list(ckpt.get_metrics()) == []  # nothing linked yet (training metrics are not "usage")
        ExperimentalCoreContext(s, infer_tid).report_task_using_checkpoint(ckpt)
        got = list(ckpt.get_metrics("inference"))
        assert [(m.trial_id, m.metrics, m.group) for m in got] == [(infer_tid, {"accuracy": 0.75}, "inference")]
        assert list(ckpt.get_metrics("validation")) == []
        model = client.create_model("src-model")
        mv = model.register_version(ck)
        assert list(mv.get_metrics()) == []
        ExperimentalCoreContext(s, infer_tid).report_task_using_model_version(mv)
        assert [m.metrics for m in mv.get_metrics("inference")] == [{"accuracy": 0.75}]
    finally:
        client.logout()
        srv.stop()
        srv.master.close()
