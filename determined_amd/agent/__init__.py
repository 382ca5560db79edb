"""The agent: exposes a node's slots to the master and runs tasks on them
(reference: ``agent/`` in Go, which launches Docker containers).

On an MI355X node the agent owns 8 GPU slots (one per GPU, discovered from the KFD topology in
sysfs -- the agent never initialises HIP itself, so spawning task processes is safe).  By default
tasks run as process groups with ``HIP_VISIBLE_DEVICES`` set to their slots; an agent can
instead run them in Docker/Podman containers (``agent/container.py``, re-attached after an agent
restart) or front a Slurm/PBS partition or a Kubernetes namespace (``agent/backends.py``).
stdout/stderr are shipped to the master line by line; exit codes are reported back.
"""

import base64
import io
import json
import logging
import os
import pathlib
import shlex
import socket
import sys
import tarfile
import threading
import time
from typing import Any, Dict, List, Optional

from determined_amd.agent.backends import ProcessBackend, TaskHandle
from determined_amd.common.api import Session

logger = logging.getLogger("determined_amd.agent")


def detect_gpus() -> List[int]:
    """GPU ordinals from /sys/class/kfd (nodes with SIMDs); honours HIP/ROCR_VISIBLE_DEVICES."""
    ids: List[int] = []
    root = pathlib.Path("/sys/class/kfd/kfd/topology/nodes")
    if root.exists():
        gpus = []
        for node in sorted(root.iterdir(), key=lambda p: int(p.name) if p.name.isdigit() else 1 << 30):
            props = node / "properties"
            try:
                kv = dict(line.split() for line in props.read_text().splitlines() if len(line.split()) == 2)
            except OSError:
                continue
            if int(kv.get("simd_count", "0")) > 0:
                gpus.append(len(gpus))
        ids = gpus
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis:
        ids = [int(x) for x in vis.split(",") if x.strip().isdigit()]
    return ids


class _Task:
    def __init__(self, cmd: Dict[str, Any]) -> None:
        self.cmd = cmd
        self.handle: Optional[TaskHandle] = None
        self.killed = False


class Agent:
    def __init__(self, master_url: str, agent_id: Optional[str] = None, slots: Optional[int] = None,
                 gpus: Optional[List[int]] = None, work_root: Optional[str] = None, host: Optional[str] = None,
                 token: Optional[str] = None, label: str = "", backend: Any = None,
                 resource_pool: Optional[str] = None) -> None:
        self.session = Session(master_url, token=token)
        self.resource_pool = resource_pool  # None: the master's default compute pool
        self.backend = backend or ProcessBackend()
        self.agent_id = agent_id or socket.gethostname()
        if getattr(self.backend, "agent_id", None) == "":  # container labels name their agent
            self.backend.agent_id = self.agent_id
        self.gpus = detect_gpus() if gpus is None else gpus
        self.use_gpu = bool(self.gpus) and slots is None
        self.devices: List[Any] = list(self.gpus) if self.use_gpu else list(range(slots if slots is not None else 1))
        self.work_root = pathlib.Path(work_root or os.path.join("/tmp", f"det-agent-{self.agent_id}"))
        self.work_root.mkdir(parents=True, exist_ok=True)
        self.host = host or "127.0.0.1"
        self.label = label
        self.tasks: Dict[str, _Task] = {}
        # allocations whose start command arrived but whose process is not up yet: listed as running
        # from the moment the command is received, so a re-registration in between never loses them
        self._starting: set = set()
        self._stop = threading.Event()

    def register(self) -> None:
        # `running`: the allocations this agent process still runs -- after an agent restart the
        # master fails the ones it lost (their trials restart under max_restarts)
        self.session.post("/api/v1/agents/register", {"agent_id": self.agent_id, "slots": len(self.devices),
                                                      "host": self.host, "devices": self.devices,
                                                      "gpu": self.use_gpu, "label": self.label,
                                                      "resource_pool": self.resource_pool,
                                                      "running": sorted(set(self.tasks) | self._starting)})
        logger.info(f"agent {self.agent_id} registered {len(self.devices)} {'GPU' if self.use_gpu else 'CPU'} slots")

    def reattach(self) -> None:
        """Pick up the tasks a previous agent process left running (container backends): they are
        listed as running when registering, and followed to their exit like freshly launched ones
        (reference agent/internal/containers/manager.go:143 reattach)."""
        if not hasattr(self.backend, "reattach"):
            return
        for r in self.backend.reattach():
            aid = r["allocation_id"]
            if aid in self.tasks:
                continue
            t = _Task({"allocation_id": aid, "task_id": r["task_id"]})
            t.handle = r["handle"]
            self.tasks[aid] = t
            logger.info(f"re-attached to allocation {aid}")
            threading.Thread(target=self._follow, args=(t, r["task_id"], aid), daemon=True).start()

    def _follow(self, t: _Task, task_id: str, aid: str) -> None:
        code = -1
        try:
            self._pump_logs(t, task_id, aid)
            assert t.handle is not None
            code = t.handle.wait()
        except Exception:
            logger.exception(f"following re-attached task {aid} failed")
        finally:
            self._report_exit(aid, code)

    def _report_exit(self, aid: str, code: int) -> None:
        self.tasks.pop(aid, None)
        try:
            self.session.post(f"/api/v1/agents/{self.agent_id}/events",
                              {"type": "exited", "allocation_id": aid, "exit_code": code})
        except Exception as e:
            logger.warning(f"could not report exit of {aid}: {e}")

    def run(self) -> None:
        self.reattach()
        self.register()
        while not self._stop.is_set():
            try:
                cmds = self.session.get(f"/api/v1/agents/{self.agent_id}/work", params={"timeout_seconds": 10},
                                        timeout=40)["commands"]
            except Exception as e:  # master restart / network blip: re-register
                logger.warning(f"agent poll failed: {e}")
                time.sleep(1)
                try:
                    self.register()
                except Exception:
                    pass
                continue
            for c in cmds:
                if c["type"] == "start":
                    self._starting.add(c["allocation_id"])
                    threading.Thread(target=self._run_task, args=(c,), daemon=True).start()
                elif c["type"] == "kill":
                    self._kill(c["allocation_id"])

    def stop(self) -> None:
        self._stop.set()
        for aid in list(self.tasks):
            self._kill(aid)

    # -- task execution ----------------------------------------------------------------------
    def _prepare_workdir(self, c: Dict[str, Any]) -> pathlib.Path:
        wd = self.work_root / c["allocation_id"]
        wd.mkdir(parents=True, exist_ok=True)
        b64 = None
        if c.get("model_def_url"):
            b64 = self.session.get(c["model_def_url"]).get("b64_tgz")
        elif c.get("workdir_b64"):
            b64 = c["workdir_b64"]
        if b64:
            with tarfile.open(fileobj=io.BytesIO(base64.b64decode(b64)), mode="r:gz") as tf:
                tf.extractall(wd, filter="data")
        return wd

    @staticmethod
    def _command(c: Dict[str, Any]) -> List[str]:
        if c.get("command"):
            cmd = c["command"]
            return ["bash", "-c", cmd] if isinstance(cmd, str) else list(cmd)
        ep = c.get("entrypoint")
        if isinstance(ep, list):
            return list(ep)
        if ep and ":" in ep and " " not in ep.strip():
            if int(c.get("slots_per_trial", 1)) > 1:
                return [sys.executable, "-m", "determined_amd.launch.torch_distributed", "--trial", ep]
            return [sys.executable, "-m", "determined_amd.exec.harness", ep]
        if ep:
            return ["bash", "-c", ep]
        raise ValueError("task has neither an entrypoint nor a command")

    def _run_task(self, c: Dict[str, Any]) -> None:
        aid = c["allocation_id"]
        t = _Task(c)
        self.tasks[aid] = t
        self._starting.discard(aid)
        code = -1
        try:
            wd = self._prepare_workdir(c)
            # the task's own variables; a process backend layers them over the agent's environment,
            # batch / pod backends ship only these
            env = {k: str(v) for k, v in c.get("env", {}).items()}
            env["DET_MODEL_DEF_DIR"] = str(wd)
            env["PYTHONPATH"] = os.pathsep.join([str(wd), _repo_root()] +
                                                [p for p in [os.environ.get("PYTHONPATH")] if p])
            env["HSA_ENABLE_IPC_MODE_LEGACY"] = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            devices = c.get("devices", [])
            if c.get("gpu"):
                if self.backend.sets_visible_devices:
                    env["HIP_VISIBLE_DEVICES"] = ",".join(str(d) for d in devices)
            else:
                env["DET_CPU_SLOTS"] = str(len(devices))
            argv = self._command(c)
            self.session.post(f"/api/v1/agents/{self.agent_id}/events", {"type": "started", "allocation_id": aid})
            t.handle = self.backend.launch(argv, wd, env, c)
            if t.killed:  # a kill raced the launch
                t.handle.kill()
            self._pump_logs(t, c["task_id"], aid)
            code = t.handle.wait()
        except Exception as e:
            logger.exception(f"task {aid} failed to run")
            self._ship(c["task_id"], aid, [f"agent: task failed to start: {e!r}"])
        finally:
            self._report_exit(aid, code)

    def _pump_logs(self, t: _Task, task_id: str, aid: str) -> None:
        """Ship log lines in batches (<= 200 lines or 0.5 s old); a flusher thread sends a partial
        batch when the task goes quiet, so the last line before a long silence is not held back."""
        assert t.handle is not None
        buf: List[str] = []
        lock = threading.Lock()
        done = threading.Event()

        def flush() -> None:
            with lock:  # held while shipping: batches reach the master in order
                if buf:
                    self._ship(task_id, aid, buf[:])
                    buf.clear()

        def flusher() -> None:
            while not done.wait(0.5):
                flush()

        threading.Thread(target=flusher, daemon=True).start()
        try:
            for line in t.handle.lines():
                with lock:
                    buf.append(line)
                    full = len(buf) >= 200
                if full:
                    flush()
        finally:
            done.set()
            flush()

    def _ship(self, task_id: str, aid: str, lines: List[str]) -> None:
        logs = []
        for ln in lines:
            rank = None
            if ln.startswith("[rank=") and "]" in ln:
                try:
                    rank = int(ln[6:ln.index("]")])
                except ValueError:
                    pass
            logs.append({"rank": rank, "log": ln})
        try:
            self.session.post("/api/v1/task/logs", {"task_id": task_id, "allocation_id": aid, "logs": logs})
        except Exception as e:
            logger.warning(f"log shipping failed: {e}")

    def _kill(self, aid: str, grace: float = 10.0) -> None:
        t = self.tasks.get(aid)
        if t is None:
            return
        t.killed = True
        if t.handle is not None:
            t.handle.kill(grace)


def _repo_root() -> str:
    return str(pathlib.Path(__file__).resolve().parents[2])
