"""Unmanaged-trial state reporting (reference ``core/_heartbeat.py``) and ``core.init(tensorboard_mode=...)``
(reference ``core/_tensorboard_mode.py``, ``core/_context.py:265-267``), against an in-process master."""

import os
import pathlib
import subprocess
import sys
import textwrap
import time

import pytest

from determined_amd.common.api import Session

ROOT = pathlib.Path(__file__).resolve().parent.parent


@pytest.fixture()
def master(tmp_path):
    from determined_amd.master import start_master

    srv = start_master()
    yield srv, f"http://127.0.0.1:{srv.port}", tmp_path
    srv.stop()
    srv.master.close()


def _defaults(core_v2, tmp_path, name):
    return core_v2.DefaultConfig(name=name, checkpoint_storage={"type": "shared_fs", "host_path": str(tmp_path)})


def _trial(url, tid):
    return Session(url).get(f"/api/v1/trials/{tid}")["trial"]


def test_unmanaged_trial_reports_completed_and_error(master):
    from determined_amd.experimental import core_v2

    srv, url, tmp = master
    ctx = core_v2.init_context(defaults=_defaults(core_v2, tmp, "ok"), master=url)
    with ctx:
        tid = ctx.info.trial.trial_id
        assert srv.master.experiments[ctx.info.trial.experiment_id].trials[1].last_activity is not None
        ctx.train.report_training_metrics(steps_completed=1, metrics={"loss": 1.0})
    assert _trial(url, tid)["state"] == "COMPLETED"

    ctx = core_v2.init_context(defaults=_defaults(core_v2, tmp, "boom"), master=url)
    with pytest.raises(ZeroDivisionError):
        with ctx:
            tid = ctx.info.trial.trial_id
            1 / 0
    assert _trial(url, tid)["state"] == "ERROR"


def test_crashed_unmanaged_process_is_marked_error(master):
    """An uncaught exception after core_v2.init(): the atexit close sees it through the exit hook."""
    _, url, tmp = master
    script = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {str(ROOT)!r})
        from determined_amd.experimental import core_v2
        core_v2.init(defaults=core_v2.DefaultConfig(name="crash", checkpoint_storage={{"type": "shared_fs",
                     "host_path": {str(tmp)!r}}}), master={url!r})
        print(core_v2.info.trial.trial_id, flush=True)
        raise RuntimeError("trial code crashed")
    """)
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "trial code crashed" in r.stderr
    tid = int(r.stdout.split()[0])
    assert _trial(url, tid)["state"] == "ERROR"

    script_ok = script.replace('raise RuntimeError("trial code crashed")', "sys.exit(3)")
    r = subprocess.run([sys.executable, "-c", script_ok], capture_output=True, text=True, timeout=120)
    assert r.returncode == 3
    assert _trial(url, int(r.stdout.split()[0]))["state"] == "ERROR"


def test_silent_unmanaged_trial_is_reaped(master):
    """A trial that reported RUNNING and then stopped sending heartbeats (killed) ends in ERROR."""
    srv, url, tmp = master
    s = Session(url)
    exp = s.post("/api/v1/unmanaged/experiments", {"config": {
        "name": "k", "searcher": {"name": "single", "metric": "x", "max_length": {"batches": 1}},
        "checkpoint_storage": {"type": "shared_fs", "host_path": str(tmp)}}})["experiment"]
    tid = s.post(f"/api/v1/unmanaged/experiments/{exp['id']}/trials", {})["trial_id"]
    s.patch(f"/api/v1/trials/{tid}", {"state": "RUNNING"})
    m = srv.master
    m.unmanaged_timeout_s = 0.3
    s.patch(f"/api/v1/trials/{tid}", {"heartbeat": True})
    with m.lock:
        m._reap_unmanaged()
    assert _trial(url, tid)["state"] != "ERROR"  # heartbeat is fresh
    time.sleep(0.5)
    with m.lock:
        m._reap_unmanaged()
    assert _trial(url, tid)["state"] == "ERROR"
    assert s.get(f"/api/v1/experiments/{exp['id']}")["experiment"]["state"] == "ERROR"


def test_managed_trial_state_is_not_reportable(master):
    srv, url, tmp = master
    s = Session(url)
    cfg = {"name": "m", "entrypoint": "x:y", "searcher": {"name": "single", "metric": "x", "max_length": {"batches": 1}},
           "checkpoint_storage": {"type": "shared_fs", "host_path": str(tmp)}, "hyperparameters": {}}
    eid = s.post("/api/v1/experiments", {"config": cfg, "activate": True})["experiment"]["id"]
    deadline = time.time() + 10
    trials = []
    while not trials and time.time() < deadline:
        trials = s.get(f"/api/v1/experiments/{eid}/trials")["trials"]
        time.sleep(0.1)
    with pytest.raises(Exception, match="400"):
        s.patch(f"/api/v1/trials/{trials[0]['id']}", {"state": "COMPLETED"})


@pytest.mark.parametrize("mode", ["AUTO", "MANUAL"])
def test_tensorboard_mode(master, mode, monkeypatch):
    from determined_amd import core
    from determined_amd.experimental import core_v2

    _, url, tmp = master
    monkeypatch.setenv("DET_TENSORBOARD_DIR", str(tmp / "tb_local"))
    ctx = core_v2.init_context(defaults=_defaults(core_v2, tmp, f"tb-{mode}"), master=url,
                               tensorboard_mode=core.TensorboardMode(mode))
    with ctx:
        eid, tid = ctx.info.trial.experiment_id, ctx.info.trial.trial_id
        ctx.train.report_training_metrics(steps_completed=1, metrics={"loss": 0.5})
        tb_path = ctx.train.get_tensorboard_path()
        if mode == "MANUAL":
            (tb_path / "mine.txt").write_text("user artifact")
    uploaded = tmp / "tensorboard" / "experiment" / str(eid) / "trial" / str(tid)
    files = sorted(p.name for p in uploaded.rglob("*") if p.is_file()) if uploaded.exists() else []
    if mode == "AUTO":
        assert any(f.startswith("events.out.tfevents") for f in files)
    else:
        assert files == []  # nothing written, nothing uploaded automatically
        assert not any(p.name.startswith("events.out") for p in tb_path.rglob("*"))


def test_tensorboard_mode_parse():
    from determined_amd.core import TensorboardMode

    assert TensorboardMode.parse(None) is TensorboardMode.AUTO
    assert TensorboardMode.parse("manual") is TensorboardMode.MANUAL
    with pytest.raises(ValueError):
        TensorboardMode.parse("sometimes")
