"""Where an agent runs its tasks: local process groups, Slurm / PBS batch jobs, or Kubernetes pods.

The reference has three resource managers for this (``master/internal/rm/agentrm`` with Go agents
launching Docker containers, ``rm/dispatcherrm`` submitting to Slurm/PBS through an HPC launcher
service, ``rm/kubernetesrm`` creating pods).  Here the master always schedules onto agents; an
agent's *backend* decides what "start this task on these slots" means:

* :class:`ProcessBackend` -- a process group on this node with ``HIP_VISIBLE_DEVICES`` set to the
  task's GPUs (the default; one agent per MI355X node).
* :class:`SlurmBackend` / :class:`PBSBackend` -- one agent fronts a batch partition: the task
  becomes one batch job (``sbatch`` / ``qsub``) spanning ``ceil(slots / slots_per_node)`` nodes,
  one :mod:`determined_amd.agent.hpc_node` per node derives the node rank and peer addresses from
  the scheduler's environment and runs the launcher (torchrun over RCCL) there.  Job state comes
  from ``squeue``/``sacct`` (``qstat``), logs from the job's output file on the shared work
  directory, kills go through ``scancel`` (``qdel``).  Experiment-config knobs follow the
  reference schema (``slurm.{slots_per_node,gpu_type,sbatch_args}``,
  ``pbs.{slots_per_node,pbsbatch_args}``; ``schemas/expconf/v0/hpc-cluster-*.json``).
* :class:`~determined_amd.agent.container.ContainerBackend` -- each task in a Docker / Podman
  container with the experiment's image, bind mounts, devices and capabilities (the reference Go
  agent's behaviour), re-attached after an agent restart.
* :class:`KubernetesBackend` -- one pod per ``slots_per_pod`` GPUs (``amd.com/gpu`` resource)
  created through the Kubernetes REST API; the experiment's ``environment.pod_spec`` is the pod
  template (reference ``kubernetesrm/spec.go``); pods find each other through the master's
  allocation all-gather, stream logs via the pod log API and are deleted on kill.

Every backend returns a :class:`TaskHandle`: an iterator of log lines, ``wait() -> exit code``
and ``kill()``.
"""

import copy
import json
import logging
import math
import os
import pathlib
import queue
import shlex
import signal
import subprocess
import sys
import threading
import time
from typing import Any, Dict, Iterator, List, Optional

logger = logging.getLogger("determined_amd.agent.backends")

ENV_FILE = "det-env.json"
LOG_FILE = "det-job.log"
EXIT_FILE = "det-job.exit"


class TaskHandle:
    def lines(self) -> Iterator[str]:
        raise NotImplementedError

    def wait(self) -> int:
        raise NotImplementedError

    def kill(self, grace: float = 10.0) -> None:
        raise NotImplementedError


def _experiment_config(env: Dict[str, str]) -> Dict[str, Any]:
    try:
        return json.loads(env.get("DET_EXPERIMENT_CONFIG") or "{}") or {}
    except ValueError:
        return {}


def _node_layout(slots: int, per_node: int) -> (int, int):
    """(number of nodes, slots per node) for a gang of ``slots`` GPUs."""
    if slots <= 0:
        return 1, 0
    nodes = max(1, math.ceil(slots / per_node))
    if slots % nodes:
        raise ValueError(f"{slots} slots cannot be split evenly over {nodes} nodes of {per_node}")
    return nodes, slots // nodes


# ------------------------------------------------------------------------------------ processes
class _ProcessHandle(TaskHandle):
    def __init__(self, proc: subprocess.Popen) -> None:
        self.proc = proc

    def lines(self) -> Iterator[str]:
        assert self.proc.stdout is not None
        for line in self.proc.stdout:
            yield line.rstrip("\n")

    def wait(self) -> int:
        return self.proc.wait()

    def kill(self, grace: float = 10.0) -> None:
        try:
            os.killpg(self.proc.pid, signal.SIGTERM)
        except ProcessLookupError:
            return

        def hard() -> None:
            time.sleep(grace)
            if self.proc.poll() is None:
                try:
                    os.killpg(self.proc.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass

        threading.Thread(target=hard, daemon=True).start()


class ProcessBackend:
    """Tasks as local process groups on the agent's node."""

    name = "process"
    sets_visible_devices = True

    def launch(self, argv: List[str], workdir: pathlib.Path, env: Dict[str, str], cmd: Dict[str, Any]) -> TaskHandle:
        full = dict(os.environ)
        full.update(env)
        uid, gid = run_as(env)
        if uid is not None:  # the owner's linked agent user (det user link-with-agent-user)
            os.chown(workdir, uid, gid if gid is not None else -1)
        proc = subprocess.Popen(argv, cwd=workdir, env=full, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                start_new_session=True, text=True, bufsize=1, user=uid,
                                group=gid if uid is not None else None)
        return _ProcessHandle(proc)


def run_as(env: Dict[str, str]):
    """(uid, gid) a task should run as: the task owner's linked agent user when the master sent
    one (DET_AGENT_UID / DET_AGENT_GID) and this agent runs as root (it can switch users); else
    (None, None) -- the task runs as the agent's own user."""
    if "DET_AGENT_UID" not in env or not hasattr(os, "geteuid") or os.geteuid() != 0:
        return None, None
    gid = env.get("DET_AGENT_GID")
    return int(env["DET_AGENT_UID"]), (int(gid) if gid not in (None, "") else None)


# ------------------------------------------------------------------------------------ batch jobs
def _run(argv: List[str], timeout: float = 60.0) -> str:
    out = subprocess.run(argv, capture_output=True, text=True, timeout=timeout)
    if out.returncode != 0:
        raise RuntimeError(f"{' '.join(argv)} failed ({out.returncode}): {out.stderr.strip()}")
    return out.stdout


class _BatchHandle(TaskHandle):
    """A submitted batch job: follows its output file until the scheduler reports it finished."""

    def __init__(self, backend: "_BatchBackend", job_id: str, workdir: pathlib.Path) -> None:
        self.backend, self.job_id, self.workdir = backend, job_id, workdir
        self._code: Optional[int] = None
        self._killed = False

    def _finished(self) -> bool:
        if self._code is not None:
            return True
        code = self.backend.exit_code(self.job_id, self.workdir)
        if code is not None:
            self._code = code
            return True
        return False

    def lines(self) -> Iterator[str]:
        log = self.workdir / LOG_FILE
        pos, partial = 0, ""
        while True:
            done = self._finished()  # decide BEFORE reading so the last bytes are not missed
            if log.exists():
                with open(log, "r", errors="replace") as f:
                    f.seek(pos)
                    chunk = f.read()
                    pos = f.tell()
                if chunk:
                    parts = (partial + chunk).split("\n")
                    partial = parts.pop()
                    yield from parts
            if done:
                if partial:
                    yield partial
                return
            time.sleep(self.backend.poll_s)

    def wait(self) -> int:
        while not self._finished():
            time.sleep(self.backend.poll_s)
        assert self._code is not None
        return self._code

    def kill(self, grace: float = 10.0) -> None:
        self._killed = True
        try:
            self.backend.cancel(self.job_id)
        except Exception as e:  # already gone
            logger.warning(f"cancelling job {self.job_id}: {e}")


class _BatchBackend:
    name = "batch"
    sets_visible_devices = False  # the batch scheduler binds GPUs to the job
    config_key = ""

    def __init__(self, slots_per_node: int = 8, extra_args: Optional[List[str]] = None,
                 python: Optional[str] = None, poll_s: float = 2.0) -> None:
        self.slots_per_node = slots_per_node
        self.extra_args = list(extra_args or [])
        self.python = python or sys.executable
        self.poll_s = poll_s

    def _settings(self, env: Dict[str, str]) -> Dict[str, Any]:
        return _experiment_config(env).get(self.config_key) or {}

    def launch(self, argv: List[str], workdir: pathlib.Path, env: Dict[str, str], cmd: Dict[str, Any]) -> TaskHandle:
        settings = self._settings(env)
        per_node = int(settings.get("slots_per_node") or self.slots_per_node)
        slots = len(cmd.get("devices", [])) if cmd.get("gpu") else 0
        nodes, gpn = _node_layout(slots, per_node)
        task_env = dict(env)
        task_env["DET_USE_GPU"] = "1" if gpn else "0"
        task_env["DET_SLOT_IDS"] = json.dumps(list(range(gpn)) if gpn else list(range(len(cmd.get("devices", [])) or 1)))
        (workdir / ENV_FILE).write_text(json.dumps(task_env))
        for stale in (LOG_FILE, EXIT_FILE):
            (workdir / stale).unlink(missing_ok=True)
        node_cmd = [self.python, "-m", "determined_amd.agent.hpc_node", self.name, "--env-file",
                    str(workdir / ENV_FILE), "--"] + list(argv)
        script = workdir / "det-job.sh"
        script.write_text(self.script(cmd, workdir, nodes, gpn, settings, node_cmd))
        script.chmod(0o755)
        job_id = self.submit(script, workdir)
        logger.info(f"{self.name}: allocation {cmd.get('allocation_id')} -> job {job_id} ({nodes}x{gpn} GPUs)")
        return _BatchHandle(self, job_id, workdir)

    def _exit_file_code(self, workdir: pathlib.Path) -> Optional[int]:
        p = workdir / EXIT_FILE
        try:
            return int(p.read_text().strip())
        except (OSError, ValueError):
            return None

    # subclass interface
    def script(self, cmd, workdir, nodes, gpn, settings, node_cmd) -> str:  # pragma: no cover
        raise NotImplementedError

    def submit(self, script: pathlib.Path, workdir: pathlib.Path) -> str:  # pragma: no cover
        raise NotImplementedError

    def exit_code(self, job_id: str, workdir: pathlib.Path) -> Optional[int]:  # pragma: no cover
        raise NotImplementedError

    def cancel(self, job_id: str) -> None:  # pragma: no cover
        raise NotImplementedError


class SlurmBackend(_BatchBackend):
    name = "slurm"
    config_key = "slurm"

    def __init__(self, partition: Optional[str] = None, **kw: Any) -> None:
        super().__init__(**kw)
        self.partition = partition

    def script(self, cmd, workdir, nodes, gpn, settings, node_cmd) -> str:
        d = [f"--job-name=det-{cmd.get('task_id', 'task')[:48]}", f"--output={workdir / LOG_FILE}",
             "--open-mode=append", f"--nodes={nodes}", "--ntasks-per-node=1", f"--chdir={workdir}"]
        if self.partition:
            d.append(f"--partition={self.partition}")
        if gpn:
            gtype = settings.get("gpu_type")
            d.append(f"--gpus-per-node={gtype + ':' if gtype else ''}{gpn}")
        d += self.extra_args + list(settings.get("sbatch_args") or [])
        lines = ["#!/bin/bash"] + [f"#SBATCH {x}" for x in d] + [
            f"srun --kill-on-bad-exit=1 --ntasks-per-node=1 {shlex.join(node_cmd)}",
            "rc=$?",
            f"echo $rc > {shlex.quote(str(workdir / EXIT_FILE))}",
            "exit $rc",
        ]
        return "\n".join(lines) + "\n"

    def submit(self, script: pathlib.Path, workdir: pathlib.Path) -> str:
        return _run(["sbatch", "--parsable", str(script)]).strip().split(";")[0]

    def exit_code(self, job_id: str, workdir: pathlib.Path) -> Optional[int]:
        purged = False
        try:
            state = _run(["squeue", "-h", "-j", job_id, "-o", "%T"]).strip()
        except RuntimeError as e:  # purged after MinJobAge ("Invalid job id specified"): no longer queued
            state, purged = "", "invalid job id" in str(e).lower()
        if state and state.split()[0] not in ("COMPLETED", "FAILED", "CANCELLED", "TIMEOUT", "NODE_FAIL",
                                              "OUT_OF_MEMORY", "PREEMPTED", "BOOT_FAIL", "DEADLINE"):
            return None
        code = self._exit_file_code(workdir)
        if code is not None:
            return code
        try:  # the job never reached its epilogue line (cancelled / node failure): ask accounting
            acct = _run(["sacct", "-n", "-P", "-X", "-j", job_id, "-o", "State,ExitCode"]).strip().splitlines()
        except Exception:
            acct = []
        if not acct:
            return None if not (state or purged) else 1
        st, _, ec = acct[0].partition("|")
        rc = int(ec.split(":")[0] or 0) if ec else 0
        if st.startswith("CANCELLED"):
            return rc or 143
        if st in ("PENDING", "RUNNING", "COMPLETING", "CONFIGURING", "REQUEUED", "SUSPENDED"):
            return None
        return rc if (rc or st == "COMPLETED") else 1

    def cancel(self, job_id: str) -> None:
        _run(["scancel", job_id])


class PBSBackend(_BatchBackend):
    name = "pbs"
    config_key = "pbs"

    def __init__(self, queue_name: Optional[str] = None, **kw: Any) -> None:
        super().__init__(**kw)
        self.queue_name = queue_name

    def script(self, cmd, workdir, nodes, gpn, settings, node_cmd) -> str:
        d = [f"-N det-{cmd.get('task_id', 'task')[:12]}", f"-o {workdir / LOG_FILE}", "-j oe"]
        if self.queue_name:
            d.append(f"-q {self.queue_name}")
        d.append(f"-l select={nodes}" + (f":ngpus={gpn}" if gpn else ""))
        if nodes > 1:
            d.append("-l place=scatter")
        d += self.extra_args + list(settings.get("pbsbatch_args") or [])
        run = shlex.join(node_cmd)
        if nodes > 1:  # one launcher per distinct node
            run = f"pbsdsh -u -- {run}"
        lines = ["#!/bin/bash"] + [f"#PBS {x}" for x in d] + [
            f"cd {shlex.quote(str(workdir))}", run, "rc=$?",
            f"echo $rc > {shlex.quote(str(workdir / EXIT_FILE))}", "exit $rc"]
        return "\n".join(lines) + "\n"

    def submit(self, script: pathlib.Path, workdir: pathlib.Path) -> str:
        return _run(["qsub", str(script)]).strip()

    def exit_code(self, job_id: str, workdir: pathlib.Path) -> Optional[int]:
        try:
            info = json.loads(_run(["qstat", "-x", "-f", "-F", "json", job_id]))
            job = next(iter(info.get("Jobs", {}).values()), {})
        except Exception:
            job = {}
        state = job.get("job_state")
        if state and state not in ("F", "X"):  # queued / running / held / exiting
            return None
        code = self._exit_file_code(workdir)
        if code is not None:
            return code
        if "Exit_status" in job:
            rc = int(job["Exit_status"])
            return rc if rc >= 0 else 1
        return None if not job else 1

    def cancel(self, job_id: str) -> None:
        _run(["qdel", job_id])


# ------------------------------------------------------------------------------------ kubernetes
class KubernetesClient:
    """The handful of core/v1 pod calls the backend needs, over plain HTTPS (no client library)."""

    SA_DIR = pathlib.Path("/var/run/secrets/kubernetes.io/serviceaccount")

    def __init__(self, api_url: Optional[str] = None, token: Optional[str] = None, verify: Any = None) -> None:
        import requests

        if api_url is None:  # in-cluster configuration
            host, port = os.environ["KUBERNETES_SERVICE_HOST"], os.environ.get("KUBERNETES_SERVICE_PORT", "443")
            api_url = f"https://{host}:{port}"
            if token is None and (self.SA_DIR / "token").exists():
                token = (self.SA_DIR / "token").read_text().strip()
            if verify is None and (self.SA_DIR / "ca.crt").exists():
                verify = str(self.SA_DIR / "ca.crt")
        self.api = api_url.rstrip("/")
        self.s = requests.Session()
        if token:
            self.s.headers["Authorization"] = f"Bearer {token}"
        self.s.verify = True if verify is None else verify

    def _url(self, ns: str, name: str = "", sub: str = "") -> str:
        return f"{self.api}/api/v1/namespaces/{ns}/pods" + (f"/{name}" if name else "") + (f"/{sub}" if sub else "")

    def create_pod(self, ns: str, pod: Dict[str, Any]) -> Dict[str, Any]:
        r = self.s.post(self._url(ns), json=pod, timeout=30)
        r.raise_for_status()
        return r.json()

    def get_pod(self, ns: str, name: str) -> Optional[Dict[str, Any]]:
        r = self.s.get(self._url(ns, name), timeout=30)
        if r.status_code == 404:
            return None
        r.raise_for_status()
        return r.json()

    def delete_pod(self, ns: str, name: str, grace: int = 10) -> None:
        r = self.s.delete(self._url(ns, name), params={"gracePeriodSeconds": grace}, timeout=30)
        if r.status_code not in (200, 202, 404):
            r.raise_for_status()

    def follow_log(self, ns: str, name: str) -> Iterator[str]:
        with self.s.get(self._url(ns, name, "log"), params={"follow": "true"}, stream=True, timeout=None) as r:
            if r.status_code >= 400:
                return
            pending = b""
            while True:  # read1: hand over whatever arrived (iter_lines would wait for full chunks)
                data = r.raw.read1(65536) if hasattr(r.raw, "read1") else r.raw.read(1)
                if not data:
                    break
                pending += data
                *done, pending = pending.split(b"\n")
                for ln in done:
                    yield ln.decode(errors="replace")
            if pending:
                yield pending.decode(errors="replace")


def _pod_exit(pod: Optional[Dict[str, Any]]) -> Optional[int]:
    if pod is None:
        return 137  # deleted under us
    st = pod.get("status", {})
    phase = st.get("phase")
    for cs in st.get("containerStatuses", []) or []:
        term = (cs.get("state") or {}).get("terminated")
        if term is not None and phase in ("Succeeded", "Failed"):
            return int(term.get("exitCode", 1))
    if phase == "Succeeded":
        return 0
    if phase == "Failed":
        return 1
    return None


class _PodsHandle(TaskHandle):
    def __init__(self, backend: "KubernetesBackend", ns: str, names: List[str]) -> None:
        self.b, self.ns, self.names = backend, ns, names
        self._q: "queue.Queue[Optional[str]]" = queue.Queue()
        self._readers = 0
        self._code: Optional[int] = None
        for rank, name in enumerate(names):
            threading.Thread(target=self._read, args=(rank, name), daemon=True).start()
            self._readers += 1

    def _read(self, rank: int, name: str) -> None:
        try:
            while True:  # the log endpoint answers 400 until the container starts
                pod = self.b.client.get_pod(self.ns, name)
                phase = (pod or {}).get("status", {}).get("phase")
                if pod is None or phase not in ("Pending", None):
                    break
                time.sleep(self.b.poll_s)
            if pod is not None:
                for line in self.b.client.follow_log(self.ns, name):
                    self._q.put(line if len(self.names) == 1 else f"[pod={rank}] {line}")
        except Exception as e:
            self._q.put(f"agent: log stream of pod {name} ended: {e!r}")
        finally:
            self._q.put(None)

    def lines(self) -> Iterator[str]:
        open_readers = self._readers
        while open_readers:
            item = self._q.get()
            if item is None:
                open_readers -= 1
            else:
                yield item

    def wait(self) -> int:
        while self._code is None:
            codes = [_pod_exit(self.b.client.get_pod(self.ns, n)) for n in self.names]
            failed = [c for c in codes if c not in (None, 0)]
            if failed:  # one rank failed: the gang is done
                self._code = failed[0]
                self.kill(grace=0)
            elif all(c == 0 for c in codes):
                self._code = 0
            else:
                time.sleep(self.b.poll_s)
        return self._code

    def kill(self, grace: float = 10.0) -> None:
        for n in self.names:
            try:
                self.b.client.delete_pod(self.ns, n, int(grace))
            except Exception as e:
                logger.warning(f"deleting pod {n}: {e}")


class KubernetesBackend:
    """Tasks as pods (one per ``slots_per_pod`` GPUs) through the Kubernetes API."""

    name = "kubernetes"
    sets_visible_devices = False  # the device plugin binds amd.com/gpu devices to the pod
    CONTAINER = "determined-container"

    def __init__(self, client: KubernetesClient, namespace: str = "default", image: str = "determined-amd:latest",
                 slots_per_pod: int = 8, gpu_resource: str = "amd.com/gpu", poll_s: float = 2.0,
                 python: str = "python3") -> None:
        self.client, self.ns, self.image = client, namespace, image
        self.slots_per_pod, self.gpu_resource, self.poll_s, self.python = slots_per_pod, gpu_resource, poll_s, python

    def pod_manifest(self, name: str, rank: int, npods: int, gpn: int, argv: List[str], env: Dict[str, str],
                     cmd: Dict[str, Any]) -> Dict[str, Any]:
        cfg = _experiment_config(env)
        base = copy.deepcopy((cfg.get("environment") or {}).get("pod_spec") or {})
        base.setdefault("apiVersion", "v1")
        base.setdefault("kind", "Pod")
        meta = base.setdefault("metadata", {})
        meta["name"] = name
        meta.setdefault("labels", {}).update({"determined-amd/allocation": cmd.get("allocation_id", ""),
                                              "determined-amd/rank": str(rank)})
        spec = base.setdefault("spec", {})
        spec["restartPolicy"] = "Never"
        containers = spec.setdefault("containers", [])
        c = next((x for x in containers if x.get("name") == self.CONTAINER), None)
        if c is None:
            c = {"name": self.CONTAINER}
            containers.insert(0, c)
        image = ((cfg.get("environment") or {}).get("image") or {})
        if isinstance(image, dict):  # normalised expconf image map (cpu / cuda / rocm); MI355X pods use rocm
            image = (image.get("rocm") or image.get("gpu") or image.get("cuda")) if gpn else image.get("cpu")
        c.setdefault("image", image or self.image)
        penv = dict(env)
        penv.update({"DET_CONTAINER_RANK": str(rank), "DET_K8S_NUM_PODS": str(npods),
                     "DET_USE_GPU": "1" if gpn else "0",
                     "DET_SLOT_IDS": json.dumps(list(range(gpn)) if gpn else [0])})
        penv.pop("DET_MODEL_DEF_DIR", None)
        penv.pop("PYTHONPATH", None)
        c["env"] = [e for e in c.get("env", []) if e.get("name") not in penv] + \
            [{"name": k, "value": str(v)} for k, v in sorted(penv.items())] + \
            [{"name": "DET_POD_IP", "valueFrom": {"fieldRef": {"fieldPath": "status.podIP"}}}]
        c["command"] = [self.python, "-m", "determined_amd.agent.hpc_node", "kubernetes", "--"] + list(argv)
        c.setdefault("workingDir", "/run/determined/workdir")
        if gpn:
            res = c.setdefault("resources", {})
            res.setdefault("limits", {})[self.gpu_resource] = gpn
            res.setdefault("requests", {})[self.gpu_resource] = gpn
        return base

    def launch(self, argv: List[str], workdir: pathlib.Path, env: Dict[str, str], cmd: Dict[str, Any]) -> TaskHandle:
        slots = len(cmd.get("devices", [])) if cmd.get("gpu") else 0
        npods, gpn = _node_layout(slots, self.slots_per_pod)
        aid = "".join(ch if ch.isalnum() else "-" for ch in str(cmd.get("allocation_id", "task")).lower())
        names = [f"det-{aid}"[:58].rstrip("-") + f"-{r}" for r in range(npods)]
        created: List[str] = []
        try:
            for r, name in enumerate(names):
                self.client.create_pod(self.ns, self.pod_manifest(name, r, npods, gpn, argv, env, cmd))
                created.append(name)
        except Exception:
            for n in created:
                self.client.delete_pod(self.ns, n, 0)
            raise
        return _PodsHandle(self, self.ns, names)


def make_backend(kind: str, **kw: Any):
    if kind == "process":
        return ProcessBackend()
    if kind == "slurm":
        return SlurmBackend(**kw)
    if kind == "pbs":
        return PBSBackend(**kw)
    if kind == "kubernetes":
        client = KubernetesClient(kw.pop("api_url", None), kw.pop("token", None), kw.pop("verify", None))
        return KubernetesBackend(client, **kw)
    if kind in ("docker", "podman"):
        from determined_amd.agent.container import ContainerBackend

        return ContainerBackend(runtime=kind, **kw)
    raise ValueError(f"unknown agent backend {kind!r}")
