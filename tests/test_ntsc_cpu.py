"""Notebook / shell / TensorBoard / command tasks and master config/logs on an in-process
master + agent (reference e2e: ``e2e_tests/tests/command``, ``test_tensorboard.py``)."""

import json
import os
import subprocess
import tempfile
import threading
import time
import urllib.request

import pytest

from determined_amd.tensorboard import MetricWriter


@pytest.fixture(scope="module")
def cl():
    from determined_amd.agent import Agent
    from determined_amd.common.api import Session
    from determined_amd.master import start_master

    srv = start_master()
    url = f"http://127.0.0.1:{srv.port}"
    ag = Agent(url, "ntsc-agent", slots=2, work_root=tempfile.mkdtemp())
    threading.Thread(target=ag.run, daemon=True).start()
    yield {"url": url, "s": Session(url), "master": srv}
    ag.stop()
    srv.stop()


def _get(url):
    with urllib.request.urlopen(url, timeout=10) as r:
        return r.read().decode()


def test_event_file_parsing_and_scalar_server(tmp_path):
    from http.server import ThreadingHTTPServer

    from determined_amd.exec.tensorboard import ScalarStore, make_handler, parse_scalar_events

    w = MetricWriter(str(tmp_path / "trial" / "7"))
    for step in range(5):
        w.write("training", step, {"loss": 1.0 / (step + 1)})
    w.write("validation", 4, {"accuracy": 0.9})
    w.close()
    f = next((tmp_path / "trial" / "7").glob("events.out.tfevents.*"))
    ev = parse_scalar_events(str(f))
    assert [e[0] for e in ev] == ["loss"] * 5 + ["val_accuracy"]
    assert ev[2][2] == 2 and abs(ev[2][3] - 1 / 3) < 1e-6
    srv = ThreadingHTTPServer(("127.0.0.1", 0), make_handler(ScalarStore({"exp-1": tmp_path})))
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    base = f"http://127.0.0.1:{srv.server_address[1]}"
    try:
        assert json.loads(_get(base + "/data/runs")) == ["exp-1/trial/7"]
        pts = json.loads(_get(base + "/data/plugin/scalars/scalars?run=exp-1/trial/7&tag=loss"))
        assert [p[1] for p in pts] == [0, 1, 2, 3, 4]
        assert "<svg" in _get(base + "/") or "polyline" in _get(base + "/")
    finally:
        srv.shutdown()


def test_tensorboard_task_serves_experiment_metrics(cl, tmp_path):
    from determined_amd.cli._ntsc import _wait_proxy

    cfg = {"name": "tb", "entrypoint": "model_def:T", "hyperparameters": {},
           "searcher": {"name": "single", "metric": "loss", "max_length": {"batches": 1}},
           "checkpoint_storage": {"type": "shared_fs", "host_path": str(tmp_path)}}
    eid = cl["s"].post("/api/v1/experiments", {"config": cfg, "activate": False})["experiment"]["id"]
    w = MetricWriter(str(tmp_path / "tensorboard" / "experiment" / str(eid) / "trial" / "1"))
    w.write("training", 10, {"loss": 0.5})
    w.close()
    tid = cl["s"].post("/api/v1/tensorboards", {"experiment_ids": [eid]})["task_id"]
    t = _wait_proxy(cl["s"], tid, timeout=60)
    base = f"http://{t['proxy']['host']}:{t['proxy']['port']}"
    assert json.loads(_get(base + "/data/runs")) == [f"exp-{eid}/trial/1"]
    assert tid in [x["id"] for x in cl["s"].get("/api/v1/tensorboards")["tasks"]]
    cl["s"].post(f"/api/v1/tasks/{tid}/kill", {})


def test_shell_task_holds_slots_and_opens_in_allocation(cl):
    from determined_amd.cli._ntsc import _wait_proxy, shell_command

    tid = cl["s"].post("/api/v1/shells", {"slots": 1})["task_id"]
    t = _wait_proxy(cl["s"], tid, timeout=60)
    sc = shell_command(t)
    assert sc["argv"] == ["bash", "-i"] and sc["env"]["DET_TASK_ID"] == tid
    env = dict(os.environ, **sc["env"])
    out = subprocess.run(["bash", "-c", "echo $DET_TASK_ID:$DET_CPU_SLOTS"], env=env, capture_output=True,
                         text=True).stdout.strip()
    assert out == f"{tid}:1"
    agents = cl["s"].get("/api/v1/agents")["agents"]
    assert sum(a["used_slots"] for a in agents) >= 1
    cl["s"].post(f"/api/v1/tasks/{tid}/kill", {})
    t0 = time.time()
    while cl["s"].get(f"/api/v1/tasks/{tid}")["task"]["state"] not in ("TERMINATED", "CANCELED"):
        assert time.time() - t0 < 30
        time.sleep(0.2)


def test_notebook_reports_missing_jupyter(cl):
    from determined_amd.cli._ntsc import _wait_proxy
    from determined_amd.exec.notebook import jupyter_available

    if jupyter_available():
        pytest.skip("jupyter present")
    tid = cl["s"].post("/api/v1/notebooks", {"slots": 0})["task_id"]
    with pytest.raises(SystemExit, match="JupyterLab is not installed"):
        _wait_proxy(cl["s"], tid, timeout=60)


def test_master_config_logs_and_command_list_cli(cl, capsys):
    from determined_amd.cli import main

    assert main(["-m", cl["url"], "master", "config"]) == 0
    assert '"scheduler"' in capsys.readouterr().out
    import logging

    logging.getLogger("determined_amd.master").warning("hello from the master log ring")
    assert main(["-m", cl["url"], "master", "logs", "--tail", "50"]) == 0
    assert "hello from the master log ring" in capsys.readouterr().out
    assert main(["-m", cl["url"], "cmd", "run", "-d", "echo", "hi"]) == 0
    assert main(["-m", cl["url"], "--json", "cmd", "list"]) == 0
    assert '"COMMAND"' in capsys.readouterr().out


def test_webhooks_state_condition_slack_and_signature(cl):
    import hashlib
    import hmac
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

    got = []

    class H(BaseHTTPRequestHandler):
        def log_message(self, *_):
            pass

        def do_POST(self):
            body = self.rfile.read(int(self.headers["Content-Length"]))
            got.append((self.path, dict(self.headers), body))
            self.send_response(200)
            self.send_header("Content-Length", "0")
            self.end_headers()

    rx = ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=rx.serve_forever, daemon=True).start()
    base = f"http://127.0.0.1:{rx.server_address[1]}"
    s = cl["s"]
    s.post("/api/v1/webhooks", {"url": base + "/paused", "triggers": [
        {"trigger_type": "EXPERIMENT_STATE_CHANGE", "condition": {"state": "PAUSED"}}]})
    s.post("/api/v1/webhooks", {"url": base + "/slack", "webhook_type": "SLACK", "triggers": [
        {"trigger_type": "EXPERIMENT_STATE_CHANGE", "condition": {"state": "CANCELED"}}]})
    cfg = {"name": "hooked", "entrypoint": "model_def:T", "hyperparameters": {},
           "searcher": {"name": "single", "metric": "loss", "max_length": {"batches": 1}},
           "checkpoint_storage": {"type": "shared_fs", "host_path": tempfile.mkdtemp()}}
    eid = s.post("/api/v1/experiments", {"config": cfg, "activate": False})["experiment"]["id"]
    s.post(f"/api/v1/experiments/{eid}/kill", {})
    t0 = time.time()
    while len([g for g in got if g[0] in ("/paused", "/slack")]) < 2 and time.time() - t0 < 20:
        time.sleep(0.1)
    rx.shutdown()
    paths = [g[0] for g in got]
    assert "/paused" in paths and "/slack" in paths
    p = next(g for g in got if g[0] == "/paused")
    ev = json.loads(p[2])
    assert ev["event_type"] == "EXPERIMENT_STATE_CHANGE" and ev["experiment"]["id"] == eid
    assert ev["experiment"]["state"] == "PAUSED"
    secret = cl["master"].master.cluster_id.encode()
    want = hmac.new(secret, (p[1]["X-Determined-AMD-Timestamp"] + "." + p[2].decode()).encode(),
                    hashlib.sha256).hexdigest()
    assert p[1]["X-Determined-AMD-Signature"] == f"sha256={want}"
    slack = json.loads(next(g for g in got if g[0] == "/slack")[2])
    assert "CANCELED" in slack["blocks"][0]["text"]["text"]
    for h in s.get("/api/v1/webhooks")["webhooks"]:
        s.delete(f"/api/v1/webhooks/{h['id']}")
