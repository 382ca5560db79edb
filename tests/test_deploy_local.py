"""``det deploy local`` (reference harness/determined/deploy/local/cli.py): cluster-up/down and the
composable master-up/down, agent-up/down and logs verbs, as local processes."""

import contextlib
import io
import time

from determined_amd.common.api import Session
from tests.dist_utils import free_port


def det(*args):
    from determined_amd.cli import main

    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        rc = main(list(args))
    assert rc in (0, None), out.getvalue()
    return out.getvalue()


def _wait(fn, timeout=30.0):
    end = time.time() + timeout
    while time.time() < end:
        try:
            v = fn()
            if v:
                return v
        except Exception:
            pass
        time.sleep(0.2)
    raise AssertionError("timed out")


def test_master_and_agent_up_down_logs(tmp_path, monkeypatch):
    monkeypatch.setenv("DET_LOCAL_CLUSTER_DIR", str(tmp_path))
    port = free_port()
    url = f"http://127.0.0.1:{port}"
    try:
        assert "local master up" in det("deploy", "local", "master-up", "--master-port", str(port))
        s = Session(url)
        det("deploy", "local", "agent-up", url, "--agent-name", "cpu0", "--no-gpu", "--cpu-slots", "2")
        agents = _wait(lambda: s.get("/api/v1/agents")["agents"])
        assert agents[0]["id"] == "agent-cpu0" and agents[0]["slots"] == 2
        assert "stopped agent-cpu0" in det("deploy", "local", "agent-down", "--agent-name", "cpu0")
        log = det("deploy", "local", "logs", "--no-follow")
        assert isinstance(log, str)
        assert "local master down" in det("deploy", "local", "master-down")
        assert "no local master" in det("deploy", "local", "master-down")
        # cluster-up / cluster-down as one
        det("deploy", "local", "cluster-up", "--master-port", str(port), "--agents", "1", "--no-gpu",
            "--cpu-slots", "1")
        _wait(lambda: Session(url).get("/api/v1/agents")["agents"])
    finally:
        det("deploy", "local", "cluster-down")
