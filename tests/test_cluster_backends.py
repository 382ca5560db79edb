"""Agent task backends: Slurm / PBS batch jobs and Kubernetes pods (``agent/backends.py``,
``agent/hpc_node.py``) plus the master's allocation all-gather.

No scheduler or cluster exists in the container, so the tests put stand-ins on ``PATH``
(``sbatch``/``squeue``/``sacct``/``scancel``/``srun``, ``qsub``/``qstat``/``qdel``) that run the
submitted script as a local process group, and serve a minimal core/v1 pods API whose "pods" are
local processes.  The agent, job scripts, node wrapper and master run unmodified against them
(reference behaviour: ``master/internal/rm/dispatcherrm``, ``rm/kubernetesrm``)."""

import json
import os
import pathlib
import signal
import subprocess
import sys
import tempfile
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

ROOT = str(pathlib.Path(__file__).resolve().parents[1])

_RUNNER = r'''
import json, os, subprocess, sys
state, jid, script, out = sys.argv[1:5]
env = dict(os.environ, **json.loads(sys.argv[5]))
with open(out, "a") as f:
    rc = subprocess.call(["bash", script], stdout=f, stderr=subprocess.STDOUT, env=env)
open(os.path.join(state, jid + ".rc"), "w").write(str(rc))
'''

_SUBMIT = r'''#!{py}
import json, os, re, subprocess, sys
state = os.environ["FAKE_SCHED_DIR"]
kind = "{kind}"
script = sys.argv[-1]
text = open(script).read()
if kind == "slurm":
    out = re.search(r"^#SBATCH --output=(\S+)", text, re.M).group(1)
    extra = {{"SLURM_JOB_NODELIST": "localhost", "SLURM_NODEID": "0"}}
else:
    out = re.search(r"^#PBS -o (\S+)", text, re.M).group(1)
    extra = {{}}
n = len([f for f in os.listdir(state) if f.endswith(".pid")]) + 1
jid = str(100 + n)
extra["JOB_ID"] = jid
p = subprocess.Popen([sys.executable, os.path.join(state, "runner.py"), state, jid, script, out, json.dumps(extra)],
                     start_new_session=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
open(os.path.join(state, jid + ".pid"), "w").write(str(p.pid))
open(os.path.join(state, jid + ".script"), "w").write(text)
print(jid if kind == "slurm" else jid + ".fakepbs")
'''

_QUERY = r'''#!{py}
import json, os, sys
state = os.environ["FAKE_SCHED_DIR"]
kind = "{kind}"
args = sys.argv[1:]
jid = args[args.index("-j") + 1] if "-j" in args else args[-1].split(".")[0]
rcf = os.path.join(state, jid + ".rc")
cancelled = os.path.exists(os.path.join(state, jid + ".cancelled"))
done = os.path.exists(rcf) or cancelled
rc = int(open(rcf).read()) if os.path.exists(rcf) else None
name = os.path.basename(sys.argv[0])
if name == "squeue":
    print("" if done else "RUNNING")
elif name == "sacct":
    if cancelled:
        print("CANCELLED by 0|0:15")
    elif rc is not None:
        print(("COMPLETED" if rc == 0 else "FAILED") + f"|{{rc}}:0")
elif name == "qstat":
    job = {{"job_state": "F", "Exit_status": -1 if cancelled and rc is None else (rc if rc is not None else 0)}} \
        if done else {{"job_state": "R"}}
    print(json.dumps({{"Jobs": {{jid + ".fakepbs": job}}}}))
'''

_CANCEL = r'''#!{py}
import os, signal, sys
state = os.environ["FAKE_SCHED_DIR"]
jid = sys.argv[-1].split(".")[0]
open(os.path.join(state, jid + ".cancelled"), "w").write("1")
try:
    os.killpg(int(open(os.path.join(state, jid + ".pid")).read()), signal.SIGTERM)
except ProcessLookupError:
    pass
'''

_SRUN = r'''#!{py}
import os, sys
args = sys.argv[1:]
while args and args[0].startswith("--"):
    args.pop(0)
os.execvp(args[0], args)
'''


@pytest.fixture()
def fake_sched(tmp_path, monkeypatch):
    state = tmp_path / "sched"
    bindir = tmp_path / "bin"
    state.mkdir()
    bindir.mkdir()
    (state / "runner.py").write_text(_RUNNER)
    py = sys.executable
    tools = {"sbatch": _SUBMIT.format(py=py, kind="slurm"), "qsub": _SUBMIT.format(py=py, kind="pbs"),
             "squeue": _QUERY.format(py=py, kind="slurm"), "sacct": _QUERY.format(py=py, kind="slurm"),
             "qstat": _QUERY.format(py=py, kind="pbs"), "scancel": _CANCEL.format(py=py),
             "qdel": _CANCEL.format(py=py), "srun": _SRUN.format(py=py)}
    for name, text in tools.items():
        (bindir / name).write_text(text)
        (bindir / name).chmod(0o755)
    monkeypatch.setenv("PATH", f"{bindir}{os.pathsep}{os.environ['PATH']}")
    monkeypatch.setenv("FAKE_SCHED_DIR", str(state))
    monkeypatch.setenv("PYTHONPATH", ROOT)  # the package is installed on the compute nodes
    return state


def _cluster(backend, slots=2):
    from determined_amd.agent import Agent
    from determined_amd.common.api import Session
    from determined_amd.master import start_master

    srv = start_master()
    url = f"http://127.0.0.1:{srv.port}"
    ag = Agent(url, f"{backend.name}-agent", slots=slots, work_root=tempfile.mkdtemp(), backend=backend)
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


# ------------------------------------------------------------------------------- unit level
def test_expand_hostlist():
    from determined_amd.agent.hpc_node import expand_hostlist

    assert expand_hostlist("gpu[01-03,07],login1") == ["gpu01", "gpu02", "gpu03", "gpu07", "login1"]
    assert expand_hostlist("n[8-10]-ib") == ["n8-ib", "n9-ib", "n10-ib"]
    assert expand_hostlist("single") == ["single"]


def test_slurm_and_pbs_scripts_span_nodes(tmp_path):
    from determined_amd.agent.backends import PBSBackend, SlurmBackend, _node_layout

    assert _node_layout(16, 8) == (2, 8) and _node_layout(4, 8) == (1, 4) and _node_layout(0, 8) == (1, 0)
    assert _node_layout(12, 8) == (2, 6)
    with pytest.raises(ValueError):
        _node_layout(9, 8)
    cmd = {"task_id": "trial-1", "allocation_id": "trial-1.1", "gpu": True, "devices": list(range(16))}
    node_cmd = ["python3", "-m", "determined_amd.agent.hpc_node", "slurm", "--", "train.py", "--lr", "0.1 x"]
    s = SlurmBackend(partition="mi355x").script(cmd, tmp_path, 2, 8, {"gpu_type": "mi355x", "sbatch_args":
                                                                     ["--time=01:00:00"]}, node_cmd)
    assert "#SBATCH --nodes=2" in s and "#SBATCH --gpus-per-node=mi355x:8" in s
    assert "#SBATCH --partition=mi355x" in s and "#SBATCH --time=01:00:00" in s
    assert "srun --kill-on-bad-exit=1 --ntasks-per-node=1 python3 -m determined_amd.agent.hpc_node" in s
    assert "'0.1 x'" in s
    p = PBSBackend().script(cmd, tmp_path, 2, 8, {"pbsbatch_args": ["-l walltime=1:00:00"]}, node_cmd)
    assert "#PBS -l select=2:ngpus=8" in p and "#PBS -l place=scatter" in p and "pbsdsh -u -- " in p
    assert "#PBS -l walltime=1:00:00" in p


def test_hpc_node_layouts(tmp_path, monkeypatch):
    from determined_amd.agent import hpc_node

    monkeypatch.setattr(hpc_node, "_resolve", lambda h: {"a1": "10.0.0.1", "a2": "10.0.0.2"}.get(h, h))
    assert hpc_node.slurm_layout({"SLURM_JOB_NODELIST": "a[1-2]", "SLURM_NODEID": "1"}) == (1, ["10.0.0.1",
                                                                                           "10.0.0.2"])
    nf = tmp_path / "nodes"
    nf.write_text("a1\na1\na2\na2\n")
    monkeypatch.setattr(hpc_node.socket, "gethostname", lambda: "a2.cluster")
    assert hpc_node.pbs_layout({"PBS_NODEFILE": str(nf)}) == (1, ["10.0.0.1", "10.0.0.2"])


def test_node_wrapper_sets_rendezvous_env(tmp_path):
    envf = tmp_path / "env.json"
    envf.write_text(json.dumps({"DET_SLOT_IDS": "[0, 1]", "FOO": "bar"}))
    code = "import os; print(os.environ['DET_CONTAINER_RANK'], os.environ['DET_CONTAINER_ADDRS'], os.environ['FOO'])"
    env = dict(os.environ, PYTHONPATH=ROOT, SLURM_JOB_NODELIST="127.0.0.1", SLURM_NODEID="0")
    out = subprocess.run([sys.executable, "-m", "determined_amd.agent.hpc_node", "slurm", "--env-file", str(envf),
                          "--", sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    assert out.stdout.split() == ["0", '["127.0.0.1"]', "bar"]
    bad = subprocess.run([sys.executable, "-m", "determined_amd.agent.hpc_node", "slurm", "--env-file", str(envf),
                          "--", sys.executable, "-c", "raise SystemExit(7)"], env=env)
    assert bad.returncode == 7


def test_master_allocation_all_gather():
    from determined_amd.common.api import Session
    from determined_amd.master import start_master

    srv = start_master()
    s = Session(f"http://127.0.0.1:{srv.port}")
    try:
        tid = s.post("/api/v1/commands", {"command": ["sleep", "30"], "slots": 0})["task_id"]
        aid = f"{tid}.1"
        out = {}

        def peer(r, rnd=0):
            out[r] = s.post(f"/api/v1/allocations/{aid}/all_gather",
                            {"request_uuid": f"u{r}-{rnd}", "num_peers": 3, "rank": r,
                             "data": f"10.{rnd}.0.{r}"})["data"]

        ts = [threading.Thread(target=peer, args=(r,)) for r in (2, 0, 1)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(30)
        assert out == {r: ["10.0.0.0", "10.0.0.1", "10.0.0.2"] for r in range(3)}
        # a retried post of a finished round (its response lost) re-fetches that round's result
        # at once and does not disturb the next round, which is forming meanwhile
        t1 = threading.Thread(target=peer, args=(1, 1))
        t1.start()
        time.sleep(0.3)
        again = s.post(f"/api/v1/allocations/{aid}/all_gather",
                       {"request_uuid": "u0-0", "num_peers": 3, "rank": 0, "data": "10.0.0.0",
                        "timeout_seconds": 2})["data"]
        assert again == ["10.0.0.0", "10.0.0.1", "10.0.0.2"]
        # the second round on the same allocation fills with new uuids
        ts = [threading.Thread(target=peer, args=(r, 1)) for r in (0, 2)]
        for t in ts:
            t.start()
        for t in ts + [t1]:
            t.join(30)
        assert out == {r: ["10.1.0.0", "10.1.0.1", "10.1.0.2"] for r in range(3)}
        with pytest.raises(Exception):
            s.post(f"/api/v1/allocations/{aid}/all_gather", {"request_uuid": "x", "num_peers": 2, "data": 1,
                                                              "timeout_seconds": 0.5})
    finally:
        srv.stop()


# ------------------------------------------------------------------------------- batch e2e
@pytest.mark.parametrize("kind", ["slurm", "pbs"])
def test_batch_backend_runs_and_kills_tasks(fake_sched, kind):
    from determined_amd.agent.backends import make_backend

    backend = make_backend(kind, poll_s=0.2)
    srv, ag, s = _cluster(backend)
    try:
        tid = s.post("/api/v1/commands", {"command": "echo hello from $DET_TASK_ID; echo rank=$DET_CONTAINER_RANK; "
                                                     "exit 3", "slots": 1})["task_id"]
        t = _wait_task(s, tid)
        assert t["exit_code"] == 3
        logs = _logs(s, tid)
        assert f"hello from {tid}" in logs and "rank=0" in logs
        scripts = [f for f in os.listdir(fake_sched) if f.endswith(".script")]
        assert len(scripts) == 1
        tid = s.post("/api/v1/commands", {"command": "echo started; sleep 60", "slots": 1})["task_id"]
        deadline = time.time() + 30
        while "started" not in _logs(s, tid) and time.time() < deadline:
            time.sleep(0.2)
        s.post(f"/api/v1/tasks/{tid}/kill", {})
        t = _wait_task(s, tid, timeout=30)
        assert t["state"] == "CANCELED" and t["exit_code"] != 0
    finally:
        ag.stop()
        srv.stop()


# ------------------------------------------------------------------------------- kubernetes
class _FakeKube:
    """core/v1 pods: create / get / delete / log?follow=true; pods are local process groups."""

    def __init__(self, root: pathlib.Path) -> None:
        self.root = root
        self.pods = {}
        self.created = []
        fk = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.0"

            def log_message(self, *a):
                pass

            def _json(self, code, obj):
                body = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_POST(self):
                assert self.headers.get("Authorization") == "Bearer t0ken"
                pod = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
                fk.start(pod)
                self._json(201, pod)

            def do_GET(self):
                path = self.path.split("?")[0]
                parts = path.strip("/").split("/")
                name = parts[5] if len(parts) > 5 else None
                p = fk.pods.get(name)
                if p is None:
                    return self._json(404, {"kind": "Status", "code": 404})
                if len(parts) > 6 and parts[6] == "log":
                    self.send_response(200)
                    self.send_header("Content-Type", "text/plain")
                    self.end_headers()
                    pos = 0
                    while True:
                        done = p["proc"].poll() is not None
                        data = p["log"].read_bytes()[pos:]
                        pos += len(data)
                        if data:
                            self.wfile.write(data)
                            self.wfile.flush()
                        if done:
                            return
                        time.sleep(0.05)
                rc = p["proc"].poll()
                status = {"phase": "Running", "podIP": "127.0.0.1"}
                if rc is not None:
                    status["phase"] = "Succeeded" if rc == 0 else "Failed"
                    status["containerStatuses"] = [{"name": "determined-container",
                                                    "state": {"terminated": {"exitCode": rc}}}]
                self._json(200, dict(p["manifest"], status=status))

            def do_DELETE(self):
                name = self.path.split("?")[0].strip("/").split("/")[5]
                p = fk.pods.pop(name, None)
                if p is not None:
                    try:
                        os.killpg(p["proc"].pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
                self._json(200, {})

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def start(self, pod):
        name = pod["metadata"]["name"]
        c = pod["spec"]["containers"][0]
        env = dict(os.environ, PYTHONPATH=ROOT)
        for e in c.get("env", []):
            env[e["name"]] = e.get("value", "127.0.0.1")  # valueFrom status.podIP
        wd = self.root / name
        wd.mkdir(parents=True, exist_ok=True)
        log = wd / "log"
        f = open(log, "wb")
        proc = subprocess.Popen(c["command"], cwd=wd, env=env, stdout=f, stderr=subprocess.STDOUT,
                                start_new_session=True)
        self.pods[name] = {"manifest": pod, "proc": proc, "log": log}
        self.created.append(pod)

    def stop(self):
        for p in self.pods.values():
            try:
                os.killpg(p["proc"].pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
        self.srv.shutdown()


def test_pod_manifest_merges_pod_spec():
    from determined_amd.agent.backends import KubernetesBackend, KubernetesClient

    b = KubernetesBackend(KubernetesClient("http://k8s.invalid", token="t"), namespace="ml", slots_per_pod=8)
    cfg = {"environment": {"image": {"gpu": "registry/det-amd:gpu", "cpu": "registry/det-amd:cpu"},
                           "pod_spec": {"metadata": {"labels": {"team": "vision"}},
                                        "spec": {"nodeSelector": {"gpu": "mi355x"},
                                                 "containers": [{"name": "determined-container",
                                                                 "volumeMounts": [{"name": "data",
                                                                                   "mountPath": "/data"}]},
                                                                {"name": "sidecar", "image": "busybox"}]}}}}
    env = {"DET_EXPERIMENT_CONFIG": json.dumps(cfg), "DET_ALLOCATION_ID": "a.1", "DET_MODEL_DEF_DIR": "/x"}
    pod = b.pod_manifest("det-a-1-1", 1, 2, 8, ["python3", "train.py"], env, {"allocation_id": "a.1"})
    assert pod["metadata"]["labels"] == {"team": "vision", "determined-amd/allocation": "a.1",
                                         "determined-amd/rank": "1"}
    assert pod["spec"]["nodeSelector"] == {"gpu": "mi355x"} and pod["spec"]["restartPolicy"] == "Never"
    c = pod["spec"]["containers"][0]
    assert c["image"] == "registry/det-amd:gpu" and c["volumeMounts"][0]["mountPath"] == "/data"
    assert c["resources"]["limits"]["amd.com/gpu"] == 8
    assert c["command"][:5] == ["python3", "-m", "determined_amd.agent.hpc_node", "kubernetes", "--"]
    names = {e["name"]: e.get("value") for e in c["env"]}
    assert names["DET_CONTAINER_RANK"] == "1" and names["DET_K8S_NUM_PODS"] == "2"
    assert "DET_MODEL_DEF_DIR" not in names and "DET_POD_IP" in names
    assert pod["spec"]["containers"][1]["name"] == "sidecar"


def test_kubernetes_backend_runs_and_kills_pods(tmp_path):
    from determined_amd.agent.backends import make_backend

    kube = _FakeKube(tmp_path / "pods")
    backend = make_backend("kubernetes", api_url=kube.url, token="t0ken", namespace="ml", poll_s=0.2,
                           python=sys.executable)
    srv, ag, s = _cluster(backend)
    try:
        tid = s.post("/api/v1/commands", {"command": "echo pod says hi; echo ip=$DET_CONTAINER_ADDRS; exit 5",
                                          "slots": 1})["task_id"]
        t = _wait_task(s, tid)
        assert t["exit_code"] == 5
        logs = _logs(s, tid)
        assert "pod says hi" in logs and 'ip=["127.0.0.1"]' in logs
        assert kube.created[0]["metadata"]["namespace"] if "namespace" in kube.created[0]["metadata"] else True
        tid = s.post("/api/v1/commands", {"command": "echo started; sleep 60", "slots": 1})["task_id"]
        deadline = time.time() + 30
        while "started" not in _logs(s, tid) and time.time() < deadline:
            time.sleep(0.2)
        s.post(f"/api/v1/tasks/{tid}/kill", {})
        t = _wait_task(s, tid, timeout=30)
        assert t["state"] == "CANCELED" and t["exit_code"] != 0
        assert not kube.pods  # deleted
    finally:
        ag.stop()
        srv.stop()
        kube.stop()


def test_hpc_config_sections_validate():
    from determined_amd import config

    base = {"entrypoint": "m:T", "hyperparameters": {},
            "searcher": {"name": "single", "metric": "loss", "max_length": {"batches": 1}}}
    ok = config.parse(dict(base, slurm={"slots_per_node": 8, "gpu_type": "mi355x", "sbatch_args": ["-t 60"]},
                           pbs={"pbsbatch_args": ["-l walltime=1:00:00"]}))
    assert ok["slurm"]["slots_per_node"] == 8 and ok["pbs"]["slots_per_node"] is None
    errs = config.validate(config.apply_defaults(dict(base, slurm={"slots_per_node": 0, "bogus": 1},
                                                      pbs={"pbsbatch_args": "nope"})))
    assert any("slurm.bogus" in e for e in errs) and any("slurm.slots_per_node" in e for e in errs)
    assert any("pbs.pbsbatch_args" in e for e in errs)


def test_slurm_exit_code_after_squeue_purged_the_job(tmp_path, monkeypatch):
    """Slurm forgets finished jobs after MinJobAge: squeue then fails with 'Invalid job id'; the
    exit file (or accounting) still gives the task's exit code instead of crashing the poll."""
    from determined_amd.agent import backends

    def fake_run(argv, timeout=60.0):
        if argv[0] == "squeue":
            raise RuntimeError("squeue -h -j 7 -o %T failed (1): slurm_load_jobs error: Invalid job id specified")
        if argv[0] == "sacct":
            return ""
        raise AssertionError(argv)

    monkeypatch.setattr(backends, "_run", fake_run)
    b = backends.SlurmBackend()
    assert b.exit_code("7", tmp_path) == 1  # purged, no exit file, no accounting: failed
    (tmp_path / backends.EXIT_FILE).write_text("3\n")
    assert b.exit_code("7", tmp_path) == 3
