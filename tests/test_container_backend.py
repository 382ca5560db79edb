"""Container agent backend (``agent/container.py``) against a stand-in ``docker`` CLI.

No container runtime exists in the container, so a fake ``docker`` on PATH records every argv and
runs ``run -d`` commands as local process groups: bind mounts are emulated by rewriting each mount
target to its source in the command and environment, ``logs -f`` / ``wait`` / ``stop`` / ``rm`` /
``ps --filter label=`` work on that state.  The agent, master and backend run unmodified against it
(reference behaviour: ``agent/pkg/docker/docker.go:244,293``,
``agent/internal/containers/manager.go:76,143,196``)."""

import json
import os
import pathlib
import signal
import subprocess
import sys
import tempfile
import threading
import time

import pytest

ROOT = str(pathlib.Path(__file__).resolve().parents[1])

_FAKE_DOCKER = r'''#!{py}
import json, os, signal, subprocess, sys, time
state = os.environ["FAKE_DOCKER_DIR"]
args = sys.argv[1:]
with open(os.path.join(state, "argv.jsonl"), "a") as f:
    f.write(json.dumps(args) + "\n")
sub = args[0]
VALUED = {{"--name", "--label", "--network", "--shm-size", "--device", "--group-add", "--security-opt", "--cap-add",
          "--cap-drop", "--mount", "-w", "-e", "--user"}}

def cdir(cid):
    return os.path.join(state, "c-" + cid)

def running(cid):
    return not os.path.exists(os.path.join(cdir(cid), "rc"))

if sub == "run":
    i, labels, mounts, envk, wd, name = 2, {{}}, [], [], None, None
    while args[i].startswith("-"):
        flag, val = args[i], args[i + 1]
        i += 2
        if flag == "--label":
            k, _, v = val.partition("=")
            labels[k] = v
        elif flag == "--mount":
            kv = dict(x.split("=", 1) if "=" in x else (x, "1") for x in val.split(","))
            mounts.append((kv["target"], kv["source"]))
        elif flag == "-e":
            envk.append(val)
        elif flag == "-w":
            wd = val
        elif flag == "--name":
            name = val
    image, cmd = args[i], args[i + 1:]
    def host(s):
        for tgt, src in sorted(mounts, key=lambda m: -len(m[0])):
            s = s.replace(tgt, src)
        return s
    env = dict(os.environ)
    env.update({{k: host(os.environ.get(k, "")) for k in envk}})
    cid = "%012x" % (len(os.listdir(state)) + 0xabc000)
    os.makedirs(cdir(cid))
    json.dump({{"labels": labels, "image": image, "name": name}}, open(os.path.join(cdir(cid), "meta.json"), "w"))
    log = open(os.path.join(cdir(cid), "log"), "w")
    # the "container init": forwards SIGTERM to the command, records its exit status like docker (128+sig)
    runner = ("import signal,subprocess,sys,os\n"
              "p=subprocess.Popen(sys.argv[2:],stdout=open(sys.argv[1]+'/log','a'),stderr=subprocess.STDOUT,"
              "start_new_session=True)\n"
              "signal.signal(signal.SIGTERM,lambda *a:os.killpg(p.pid,signal.SIGTERM))\n"
              "rc=p.wait()\nrc=128-rc if rc<0 else rc\n"
              "open(sys.argv[1]+'/rc.tmp','w').write(str(rc))\nos.rename(sys.argv[1]+'/rc.tmp',sys.argv[1]+'/rc')")
    p = subprocess.Popen([sys.executable, "-c", runner, cdir(cid)] + [host(c) for c in cmd], cwd=host(wd or "/"),
                         env=env, start_new_session=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    open(os.path.join(cdir(cid), "pid"), "w").write(str(p.pid))
    print(cid)
elif sub == "logs":
    cid = args[-1]
    pos = 0
    while True:
        done = not running(cid)
        with open(os.path.join(cdir(cid), "log")) as f:
            f.seek(pos)
            chunk = f.read()
            pos = f.tell()
        sys.stdout.write(chunk)
        sys.stdout.flush()
        if done:
            break
        time.sleep(0.05)
elif sub == "wait":
    cid = args[-1]
    while running(cid):
        time.sleep(0.05)
    print(open(os.path.join(cdir(cid), "rc")).read())
elif sub in ("stop", "rm"):
    cid = args[-1]
    if os.path.isdir(cdir(cid)) and running(cid):
        try:
            os.killpg(int(open(os.path.join(cdir(cid), "pid")).read()), signal.SIGTERM)
        except ProcessLookupError:
            pass
    if sub == "rm" and os.path.isdir(cdir(cid)):
        open(os.path.join(cdir(cid), "removed"), "w").write("1")
elif sub == "ps":
    want = args[args.index("--filter") + 1].split("=", 1)[1]
    wk, _, wv = want.partition("=")
    for d in sorted(os.listdir(state)):
        if not d.startswith("c-") or os.path.exists(os.path.join(state, d, "removed")):
            continue
        meta = json.load(open(os.path.join(state, d, "meta.json")))
        if meta["labels"].get(wk) == wv:
            lab = meta["labels"]
            print("\t".join([d[2:], lab.get("determined-amd.allocation", ""), lab.get("determined-amd.task", "")]))
elif sub in ("pull", "login"):
    if sub == "login":
        open(os.path.join(state, "login-stdin"), "w").write(sys.stdin.read())
else:
    sys.exit("fake docker: unsupported " + sub)
'''


@pytest.fixture()
def fake_docker(tmp_path, monkeypatch):
    state = tmp_path / "docker"
    bindir = tmp_path / "bin"
    state.mkdir()
    bindir.mkdir()
    (bindir / "docker").write_text(_FAKE_DOCKER.format(py=sys.executable))
    (bindir / "docker").chmod(0o755)
    monkeypatch.setenv("PATH", f"{bindir}{os.pathsep}{os.environ['PATH']}")
    monkeypatch.setenv("FAKE_DOCKER_DIR", str(state))
    return state


def _argvs(state):
    return [json.loads(ln) for ln in (state / "argv.jsonl").read_text().splitlines()]


def _topology(tmp_path, minors):
    root = tmp_path / "topo"
    (root / "0").mkdir(parents=True)
    (root / "0" / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    for i, m in enumerate(minors, start=1):
        (root / str(i)).mkdir()
        (root / str(i) / "properties").write_text(f"simd_count 1024\ndrm_render_minor {m}\n")
    return str(root)


def test_run_args_honour_the_experiment_environment(tmp_path):
    from determined_amd.agent.container import PKGDIR, WORKDIR, ContainerBackend
    from determined_amd.config import apply_defaults

    cfg = apply_defaults({
        "searcher": {"name": "single", "metric": "l", "max_length": 1},
        "environment": {"image": {"cpu": "img:cpu", "rocm": "img:rocm"}, "environment_variables": ["A=1", "B=x=y"],
                        "add_capabilities": ["SYS_PTRACE"], "drop_capabilities": ["NET_RAW"]},
        "bind_mounts": [{"host_path": "/data", "container_path": "/mnt/data", "read_only": True}],
        "resources": {"shm_size": 1 << 30, "devices": ["/dev/infiniband/uverbs0:/dev/infiniband/uverbs0"]}})
    env = {"DET_EXPERIMENT_CONFIG": json.dumps(cfg), "DET_SESSION_TOKEN": "secret-token", "HIP_VISIBLE_DEVICES": "2,5"}
    be = ContainerBackend(agent_id="node1", topology=_topology(tmp_path, [128, 129, 130, 131, 132, 133]))
    cmd = {"allocation_id": "exp-1.trial-2.1", "task_id": "t-2", "gpu": True, "devices": [2, 5]}
    args, task_env, image = be.run_args([sys.executable, "-m", "x"], tmp_path, env, cmd)
    assert image == "img:rocm" and args[:3] == ["docker", "run", "-d"]
    joined = " ".join(args)
    assert "--device /dev/kfd" in joined and "--device /dev/dri/renderD130" in joined and \
        "--device /dev/dri/renderD133" in joined and "renderD128" not in joined
    assert "HIP_VISIBLE_DEVICES" not in task_env  # the container sees exactly its two GPUs
    assert "--shm-size 1073741824" in joined and "--cap-add SYS_PTRACE" in joined and "--cap-drop NET_RAW" in joined
    assert "type=bind,source=/data,target=/mnt/data,readonly,bind-propagation=rprivate" in joined
    assert f"type=bind,source={tmp_path},target={WORKDIR}" in joined and f"target={PKGDIR},readonly" in joined
    assert "--device /dev/infiniband/uverbs0:/dev/infiniband/uverbs0" in joined
    assert "--label determined-amd.agent=node1" in joined and "--network host" in joined
    assert "secret-token" not in joined and "-e DET_SESSION_TOKEN" in joined  # values stay off argv
    assert task_env["A"] == "1" and task_env["B"] == "x=y" and task_env["PYTHONPATH"] == f"{WORKDIR}:{PKGDIR}"
    assert args[args.index("img:rocm") + 1:] == ["python3", "-m", "x"]
    # CPU task: cpu image, no GPU devices; an unmappable slot falls back to /dev/dri + HIP_VISIBLE_DEVICES
    args, _, image = be.run_args(["true"], tmp_path, env, {"allocation_id": "a", "gpu": False, "devices": [0]})
    assert image == "img:cpu" and "/dev/kfd" not in args
    args, task_env, _ = be.run_args(["true"], tmp_path, env, {"allocation_id": "a", "gpu": True, "devices": [7]})
    assert "/dev/dri" in args and task_env["HIP_VISIBLE_DEVICES"] == "7"


def _cluster(backend, agent_id="docker-agent", slots=2):
    from determined_amd.agent import Agent
    from determined_amd.common.api import Session
    from determined_amd.master import start_master

    srv = start_master()
    url = f"http://127.0.0.1:{srv.port}"
    ag = Agent(url, agent_id, slots=slots, work_root=tempfile.mkdtemp(), backend=backend)
    threading.Thread(target=ag.run, daemon=True).start()
    return srv, ag, Session(url)


def _wait_task(s, tid, timeout=60):
    deadline = time.time() + timeout
    while time.time() < deadline:
        t = s.get(f"/api/v1/tasks/{tid}")["task"]
        if t["state"] in ("TERMINATED", "CANCELED"):
            return t
        time.sleep(0.2)
    raise TimeoutError(f"task {tid} did not finish")


def _logs(s, tid):
    return [x["log"] for x in s.get(f"/api/v1/tasks/{tid}/logs")["logs"]]


def test_container_backend_runs_logs_and_kills(fake_docker):
    from determined_amd.agent.backends import make_backend

    srv, ag, s = _cluster(make_backend("docker"))
    try:
        conf = {"environment": {"image": "my/image:1", "environment_variables": ["GREETING=hi"],
                                "force_pull_image": True, "registry_auth": {"username": "u", "password": "pw"}},
                "bind_mounts": [{"host_path": "/tmp", "container_path": "/scratch"}]}
        tid = s.post("/api/v1/commands", {"command": "echo $GREETING from $DET_TASK_ID in $(pwd); exit 3",
                                          "slots": 1, "config": conf})["task_id"]
        t = _wait_task(s, tid)
        assert t["exit_code"] == 3
        logs = _logs(s, tid)
        assert any(ln.startswith(f"hi from {tid} in ") for ln in logs), logs
        argvs = _argvs(fake_docker)
        subs = [a[0] for a in argvs]
        assert subs.index("login") < subs.index("pull") < subs.index("run")
        run = next(a for a in argvs if a[0] == "run")
        assert "my/image:1" in run and "type=bind,source=/tmp,target=/scratch,bind-propagation=rprivate" in run
        assert ["rm", "-f"] == next(a for a in argvs if a[0] == "rm")[:2]
        assert (fake_docker / "login-stdin").read_text() == "pw"
        tid = s.post("/api/v1/commands", {"command": "echo started; sleep 60", "slots": 1})["task_id"]
        deadline = time.time() + 30
        while "started" not in _logs(s, tid) and time.time() < deadline:
            time.sleep(0.2)
        s.post(f"/api/v1/tasks/{tid}/kill", {})
        t = _wait_task(s, tid, timeout=30)
        assert t["state"] == "CANCELED" and t["exit_code"] != 0
        assert any(a[0] == "stop" for a in _argvs(fake_docker))
    finally:
        ag.stop()
        srv.stop()


def test_agent_restart_reattaches_running_container(fake_docker, tmp_path):
    """An agent process killed with -9 leaves its container running; a new agent with the same id
    finds it by label, reports it as running when it registers (so the master keeps the allocation),
    follows its logs and reports its real exit code."""
    from determined_amd.agent import Agent
    from determined_amd.agent.backends import make_backend
    from determined_amd.common.api import Session
    from determined_amd.master import start_master

    srv = start_master()
    url = f"http://127.0.0.1:{srv.port}"
    s = Session(url)
    gate = tmp_path / "gate"
    proc = subprocess.Popen([sys.executable, "-m", "determined_amd.agent", "--master-url", url, "--agent-id", "n1",
                             "--slots", "1", "--backend", "docker", "--work-root", str(tmp_path / "w1")],
                            env=dict(os.environ, PYTHONPATH=ROOT), start_new_session=True,
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    ag = None
    try:
        tid = s.post("/api/v1/commands", {"command": f"echo before; while [ ! -e {gate} ]; do sleep 0.1; done; "
                                                     "echo after; exit 7", "slots": 1})["task_id"]
        deadline = time.time() + 60
        while "before" not in _logs(s, tid) and time.time() < deadline:
            time.sleep(0.2)
        assert "before" in _logs(s, tid)
        os.killpg(proc.pid, signal.SIGKILL)  # the agent dies; the container keeps running
        proc.wait()
        ag = Agent(url, "n1", slots=1, work_root=str(tmp_path / "w2"), backend=make_backend("docker"))
        threading.Thread(target=ag.run, daemon=True).start()
        deadline = time.time() + 30
        while "n1" not in str(ag.tasks.keys()) and not ag.tasks and time.time() < deadline:
            time.sleep(0.1)
        time.sleep(1.0)  # registered with the task listed as running
        assert s.get(f"/api/v1/tasks/{tid}")["task"]["state"] not in ("TERMINATED", "CANCELED")
        gate.write_text("go")
        t = _wait_task(s, tid, timeout=30)
        assert t["exit_code"] == 7
        assert "after" in _logs(s, tid)
    finally:
        if proc.poll() is None:
            os.killpg(proc.pid, signal.SIGKILL)
        if ag is not None:
            ag.stop()
        srv.stop()
