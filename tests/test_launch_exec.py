"""Launch/exec layer: worker supervision (pid_server/pid_client), checkpoint GC task, container
prep checks and the DeepSpeed-style launcher command (reference tests:
``harness/tests/launch/test_deepspeed.py``, ``harness/tests/test_ipc.py``)."""

import json
import os
import signal
import subprocess
import sys
import threading
import time

import pytest

from determined_amd.exec import gc_checkpoints, prep_container
from determined_amd.launch import deepspeed as ds_launch
from determined_amd.launch.supervisor import (WorkerClient, WorkerFailed, WorkerSupervisor, parse_addr,
                                              parse_signal)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONPATH=ROOT)


def test_parse_helpers():
    assert parse_addr("/tmp/x.sock") == "/tmp/x.sock"
    assert parse_addr("1234") == 1234
    assert parse_addr("10.0.0.1:99") == ("10.0.0.1", 99)
    with pytest.raises(ValueError):
        parse_addr("nope")
    assert parse_signal("wait") is None
    assert parse_signal("term") == signal.SIGTERM
    assert parse_signal("SIGKILL") == signal.SIGKILL
    with pytest.raises(ValueError):
        parse_signal("SIGFOO")


def _worker(addr, code, delay=0.05):
    c = WorkerClient(addr).start()
    time.sleep(delay)
    c.keep_alive()
    c.close(code)


def test_supervisor_all_clean(tmp_path):
    addr = str(tmp_path / "s.sock")
    with WorkerSupervisor(addr, 3) as sup:
        ts = [threading.Thread(target=_worker, args=(addr, 0)) for _ in range(3)]
        for t in ts:
            t.start()
        sup.run(poll_s=0.05)
        for t in ts:
            t.join()
    assert sup.finished and len(sup.pids) == 3


def test_supervisor_detects_failed_worker(tmp_path):
    addr = str(tmp_path / "s.sock")
    with WorkerSupervisor(addr, 2) as sup:
        ts = [threading.Thread(target=_worker, args=(addr, c)) for c in (0, 3)]
        for t in ts:
            t.start()
        with pytest.raises(WorkerFailed, match="code 3"):
            sup.run(poll_s=0.05)
        for t in ts:
            t.join()


def test_supervisor_detects_crash_without_goodbye(tmp_path):
    addr = str(tmp_path / "s.sock")
    with WorkerSupervisor(addr, 1) as sup:
        # a child process that registers and is then SIGKILLed (no goodbye)
        code = ("import time,sys; from determined_amd.launch.supervisor import WorkerClient; "
                f"c=WorkerClient({addr!r}).start(); time.sleep(30)")
        p = subprocess.Popen([sys.executable, "-c", code], env=ENV)
        t0 = time.time()
        while not sup.pids and time.time() - t0 < 30:
            for key, _ in sup.sel.select(timeout=0.1):
                if key.fileobj is sup.listener:
                    sup._accept()
                else:
                    sup._consume(key.fileobj)
        p.kill()
        p.wait()
        with pytest.raises(WorkerFailed):
            sup.run(poll_s=0.05)


def test_pid_server_signals_launcher_on_worker_failure(tmp_path):
    """pid_server runs a 'launcher' that sleeps; one of two pid_client workers fails -> the
    launcher gets SIGTERM and the server exits non-zero quickly."""
    sock = str(tmp_path / "p.sock")
    server = subprocess.Popen([sys.executable, "-m", "determined_amd.exec.pid_server", "--grace-period", "0",
                               sock, "2", "--", sys.executable, "-c", "import time; time.sleep(60)"], env=ENV)
    while not os.path.exists(sock):
        time.sleep(0.05)
    ok = subprocess.Popen([sys.executable, "-m", "determined_amd.exec.pid_client", sock, "--",
                           sys.executable, "-c", "import time; time.sleep(0.5)"], env=ENV)
    bad = subprocess.run([sys.executable, "-m", "determined_amd.exec.pid_client", sock, "--",
                          sys.executable, "-c", "import sys; sys.exit(5)"], env=ENV)
    assert bad.returncode == 5
    t0 = time.time()
    rc = server.wait(timeout=30)
    assert time.time() - t0 < 20
    assert rc != 0
    # the healthy worker may not even have registered before the failure tore the gang down
    ok.kill()
    ok.wait(timeout=30)


def test_pid_server_clean_run(tmp_path):
    sock = str(tmp_path / "p.sock")
    server = subprocess.Popen([sys.executable, "-m", "determined_amd.exec.pid_server", sock, "1", "--",
                               sys.executable, "-c", "import time; time.sleep(5.0)"], env=ENV)
    while not os.path.exists(sock):
        time.sleep(0.05)
    w = subprocess.run([sys.executable, "-m", "determined_amd.exec.pid_client", sock, "--",
                        sys.executable, "-c", "pass"], env=ENV)
    assert w.returncode == 0
    assert server.wait(timeout=30) == 0


def test_gc_checkpoints_full_and_partial(tmp_path, capsys):
    base = tmp_path / "ckpts"
    for u in ("a1", "b2"):
        (base / u / "sub").mkdir(parents=True)
        (base / u / "model.pt").write_text("x")
        (base / u / "sub" / "opt.pt").write_text("y")
        (base / u / "metadata.json").write_text("{}")
    (base / "tensorboard" / "experiment" / "7").mkdir(parents=True)
    cfg = json.dumps({"type": "shared_fs", "host_path": str(base)})
    rc = gc_checkpoints.main(["--storage-config", cfg, "--delete", '["a1"]', "--experiment-id", "7",
                              "--delete-tensorboards"])
    assert rc == 0
    assert not (base / "a1").exists()
    assert not (base / "tensorboard" / "experiment" / "7").exists()
    rc = gc_checkpoints.main(["--storage-config", cfg, "--delete", '["b2"]', "--globs", '["**/*.pt"]'])
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert (base / "b2" / "metadata.json").exists() and not (base / "b2" / "model.pt").exists()
    assert "metadata.json" in out["remaining"]["b2"]
    gc_checkpoints.main(["--storage-config", cfg, "--delete", '["b2"]', "--dry-run"])
    assert (base / "b2").exists()


def _fake_kfd(root, gpus):
    for i, (simd, hbm) in enumerate([(0, 0)] + gpus):  # node 0 is the CPU
        n = root / str(i)
        (n / "mem_banks" / "0").mkdir(parents=True)
        (n / "properties").write_text(f"simd_count {simd}\ngfx_target_version 90500\n")
        (n / "mem_banks" / "0" / "properties").write_text(f"size_in_bytes {hbm}\n")


def test_prep_container_resources(tmp_path, monkeypatch):
    _fake_kfd(tmp_path, [(1024, 288 << 30)] * 2)
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    inv = prep_container.gpu_inventory(tmp_path)
    assert [g["hbm_bytes"] for g in inv] == [288 << 30] * 2
    assert len(prep_container.check_resources([0, 1], True, tmp_path)) == 2
    with pytest.raises(RuntimeError):
        prep_container.check_resources([0, 5], True, tmp_path)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    with pytest.raises(RuntimeError):
        prep_container.check_resources([0, 1], True, tmp_path)
    assert prep_container.check_resources([0, 1], False, tmp_path) == []


def test_prep_container_rendezvous(tmp_path):
    env = {"DET_CONTAINER_ADDRS": '["127.0.0.1", "127.0.0.2"]', "DET_CONTAINER_RANK": "0",
           "DET_SLOT_IDS": "[0,1,2,3,4,5,6,7]"}
    info = prep_container.do_rendezvous(str(tmp_path / "r.json"), env)
    assert info["chief"] == "127.0.0.1" and info["num_nodes"] == 2 and info["slots_per_node"] == 8
    assert info["socket_ifname"] == "lo"
    assert json.loads((tmp_path / "r.json").read_text()) == info


def test_deepspeed_launch_cmd():
    single = ds_launch.build_cmd([], ["--trial", "model_def:T"],
                                 {"DET_SLOT_IDS": "[0,1,2,3]", "DET_USE_GPU": "1"})
    assert "pid_server" not in " ".join(single) and "pid_client" not in " ".join(single)
    assert single[single.index("--nproc-per-node") + 1] == "4"
    env = {"DET_SLOT_IDS": "[0,1,2,3,4,5,6,7]", "DET_USE_GPU": "1",
           "DET_CONTAINER_ADDRS": '["10.0.0.1", "10.0.0.2"]', "DET_CONTAINER_RANK": "0"}
    chief = ds_launch.build_cmd([], ["--trial", "model_def:T"], env)
    j = " ".join(chief)
    assert "determined_amd.exec.pid_server" in j and " 16 " in j and "10.0.0.1:" in j
    env["DET_CONTAINER_RANK"] = "1"
    other = " ".join(ds_launch.build_cmd([], ["--trial", "model_def:T"], env))
    assert "pid_server" not in other and "pid_client" in other and "--node-rank 1" in other
