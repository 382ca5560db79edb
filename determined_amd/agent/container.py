"""Container task backend: every task runs in a Docker / Podman container on the agent's node.

Reference behaviour: the Go agent creates, starts, follows and re-attaches task containers through
the Docker API (``agent/pkg/docker/docker.go:244`` CreateContainer, ``:293`` RunContainer;
``agent/internal/containers/manager.go:76`` revalidate / ``:143`` reattach, ``:196``
StartContainer).  Here the agent drives the ``docker`` (or ``podman``) CLI, which needs no client
library and behaves the same for both runtimes:

* ``run -d`` with the experiment's ``environment.image`` (``rocm`` entry for GPU tasks, ``cpu`` for
  CPU tasks), ``environment.force_pull_image`` / ``registry_auth`` (pull / login first),
  ``environment_variables`` (passed as ``-e KEY`` so values -- session tokens included -- never
  appear on a command line), ``add_capabilities`` / ``drop_capabilities``, ``bind_mounts``
  (``--mount type=bind`` with read-only and propagation), ``resources.devices`` and
  ``resources.shm_size``;
* ROCm device exposure for the allocated slots: ``/dev/kfd`` plus only the DRM render nodes of the
  task's GPUs (looked up in the KFD topology), so the container sees exactly its GPUs as 0..n-1;
  when the topology cannot map a slot the whole ``/dev/dri`` is passed and ``HIP_VISIBLE_DEVICES``
  selects the slots instead;
* host networking (rendezvous over the nodes' addresses, like the process backend), the task work
  directory mounted at ``/run/determined/workdir`` and this package mounted read-only at
  ``/run/determined/pkg``;
* ``logs -f`` for the log stream, ``wait`` for the exit code, ``stop -t <grace>`` to kill, ``rm -f``
  to clean up;
* re-attach after an agent restart: containers carry ``determined-amd.*`` labels (agent, allocation,
  task); :meth:`ContainerBackend.reattach` lists this agent's containers so the agent resumes
  following them and reports them as still running when it re-registers.
"""

import json
import logging
import os
import pathlib
import subprocess
import sys
import threading
from typing import Any, Dict, Iterator, List, Optional, Tuple

from determined_amd.agent.backends import TaskHandle, _experiment_config, run_as

logger = logging.getLogger("determined_amd.agent.container")

WORKDIR = "/run/determined/workdir"
PKGDIR = "/run/determined/pkg"
LABEL = "determined-amd"
DEFAULT_SHM = "4294967296"  # reference task_container_defaults.shm_size_bytes
DEFAULT_IMAGE = "rocm/pytorch:latest"
KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"


def render_minors(topology: str = KFD_TOPOLOGY) -> List[int]:
    """DRM render-node minors of the node's GPUs in GPU-ordinal order (KFD topology nodes with SIMDs)."""
    root = pathlib.Path(topology)
    out: List[int] = []
    if not root.exists():
        return out
    for node in sorted(root.iterdir(), key=lambda p: int(p.name) if p.name.isdigit() else 1 << 30):
        try:
            kv = dict(ln.split() for ln in (node / "properties").read_text().splitlines() if len(ln.split()) == 2)
        except OSError:
            continue
        if int(kv.get("simd_count", "0")) > 0:
            out.append(int(kv.get("drm_render_minor", "-1")))
    return out


def _task_config(env: Dict[str, str]) -> Dict[str, Any]:
    cfg = _experiment_config(env)
    if not cfg and env.get("DET_TASK_CONFIG"):
        try:
            cfg = json.loads(env["DET_TASK_CONFIG"]) or {}
        except ValueError:
            cfg = {}
    return cfg


def _image_for(image: Any, gpu: bool, default: str) -> str:
    if isinstance(image, str) and image:
        return image
    if isinstance(image, dict):
        pick = (image.get("rocm") or image.get("gpu") or image.get("cuda")) if gpu else image.get("cpu")
        if pick:
            return str(pick)
    return default


def _env_vars(ev: Any, gpu: bool) -> List[str]:
    if isinstance(ev, dict):
        ev = ev.get("rocm" if gpu else "cpu") or ev.get("gpu" if gpu else "cpu") or []
    return [str(x) for x in (ev or [])]


class _ContainerHandle(TaskHandle):
    def __init__(self, backend: "ContainerBackend", cid: str) -> None:
        self.b, self.cid = backend, cid
        self._code: Optional[int] = None
        self._lock = threading.Lock()

    def lines(self) -> Iterator[str]:
        p = subprocess.Popen(self.b.cli + ["logs", "-f", self.cid], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                             text=True, bufsize=1)
        assert p.stdout is not None
        try:
            for line in p.stdout:
                yield line.rstrip("\n")
        finally:
            p.wait()

    def wait(self) -> int:
        with self._lock:
            if self._code is None:
                out = subprocess.run(self.b.cli + ["wait", self.cid], capture_output=True, text=True)
                try:
                    self._code = int(out.stdout.strip().splitlines()[-1])
                except (ValueError, IndexError):
                    logger.warning(f"{self.b.cli[0]} wait {self.cid}: {out.stderr.strip()}")
                    self._code = 1
                if not self.b.keep:
                    subprocess.run(self.b.cli + ["rm", "-f", self.cid], capture_output=True, text=True)
            return self._code

    def kill(self, grace: float = 10.0) -> None:
        def stop() -> None:
            subprocess.run(self.b.cli + ["stop", "-t", str(int(grace)), self.cid], capture_output=True, text=True)

        threading.Thread(target=stop, daemon=True).start()


class ContainerBackend:
    """Tasks as containers through the ``docker`` / ``podman`` CLI."""

    sets_visible_devices = False  # device nodes (or HIP_VISIBLE_DEVICES when unmappable) set per task

    def __init__(self, runtime: str = "docker", default_image: str = DEFAULT_IMAGE, agent_id: str = "",
                 topology: str = KFD_TOPOLOGY, keep: bool = False, python: str = "python3",
                 pkg_root: Optional[str] = None, network: str = "host") -> None:
        self.name = runtime
        self.cli = [runtime]
        self.default_image = default_image
        self.agent_id = agent_id
        self.topology = topology
        self.keep = keep  # leave exited containers for inspection
        self.python = python
        self.pkg_root = pkg_root or str(pathlib.Path(__file__).resolve().parents[2])
        self.network = network

    # ------------------------------------------------------------------------------ argv
    def run_args(self, argv: List[str], workdir: pathlib.Path, env: Dict[str, str], cmd: Dict[str, Any]
                 ) -> Tuple[List[str], Dict[str, str], str]:
        """(docker run argv, the task environment, image) for one task."""
        cfg = _task_config(env)
        envc = cfg.get("environment") or {}
        res = cfg.get("resources") or {}
        gpu = bool(cmd.get("gpu"))
        devices = [int(d) for d in cmd.get("devices", [])] if gpu else []
        image = _image_for(envc.get("image"), gpu, self.default_image)
        aid = str(cmd.get("allocation_id", "task"))
        name = "det-" + "".join(ch if ch.isalnum() or ch in "-_." else "-" for ch in aid)
        args = self.cli + ["run", "-d", "--name", name,
                           "--label", f"{LABEL}.agent={self.agent_id}", "--label", f"{LABEL}.allocation={aid}",
                           "--label", f"{LABEL}.task={cmd.get('task_id', '')}",
                           "--network", self.network, "--shm-size", str(res.get("shm_size") or DEFAULT_SHM)]
        task_env = dict(env)
        for kv in _env_vars(envc.get("environment_variables"), gpu):
            k, _, v = kv.partition("=")
            task_env[k] = v
        # GPU exposure: /dev/kfd + the render nodes of the allocated GPUs
        if gpu:
            args += ["--device", "/dev/kfd", "--group-add", "video", "--group-add", "render",
                     "--security-opt", "seccomp=unconfined"]
            minors = render_minors(self.topology)
            if devices and all(0 <= d < len(minors) and minors[d] >= 0 for d in devices):
                for d in devices:
                    args += ["--device", f"/dev/dri/renderD{minors[d]}"]
                task_env.pop("HIP_VISIBLE_DEVICES", None)
            else:
                args += ["--device", "/dev/dri"]
                task_env["HIP_VISIBLE_DEVICES"] = ",".join(str(d) for d in devices)
        for dev in res.get("devices") or []:
            if isinstance(dev, str):
                args += ["--device", dev]
            elif isinstance(dev, dict):
                args += ["--device", f"{dev['host_path']}:{dev['container_path']}:{dev.get('mode') or 'mrw'}"]
        for cap in envc.get("add_capabilities") or []:
            args += ["--cap-add", str(cap)]
        for cap in envc.get("drop_capabilities") or []:
            args += ["--cap-drop", str(cap)]
        for bm in cfg.get("bind_mounts") or []:
            spec = f"type=bind,source={bm['host_path']},target={bm['container_path']}"
            if bm.get("read_only"):
                spec += ",readonly"
            spec += f",bind-propagation={bm.get('propagation') or 'rprivate'}"
            args += ["--mount", spec]
        args += ["--mount", f"type=bind,source={workdir},target={WORKDIR}",
                 "--mount", f"type=bind,source={self.pkg_root},target={PKGDIR},readonly", "-w", WORKDIR]
        uid, gid = run_as(env)
        if uid is not None:
            args += ["--user", f"{uid}:{gid}" if gid is not None else str(uid)]
        # paths inside the container: the work dir and the package mount replace the host's
        task_env["DET_MODEL_DEF_DIR"] = WORKDIR
        task_env["PYTHONPATH"] = f"{WORKDIR}:{PKGDIR}"
        for k in sorted(task_env):  # values travel in the CLI's environment, not on its argv
            args += ["-e", k]
        args.append(image)
        inner = list(argv)
        if inner and inner[0] == sys.executable:
            inner[0] = self.python
        args += inner
        return args, task_env, image

    # ------------------------------------------------------------------------------ lifecycle
    def _prepare_image(self, image: str, env: Dict[str, str], cli_env: Dict[str, str]) -> None:
        envc = _task_config(env).get("environment") or {}
        auth = envc.get("registry_auth") or {}
        if auth.get("username") and auth.get("password"):
            login = self.cli + ["login", "-u", auth["username"], "--password-stdin"]
            if auth.get("serveraddress"):
                login.append(auth["serveraddress"])
            out = subprocess.run(login, input=auth["password"], capture_output=True, text=True, env=cli_env)
            if out.returncode != 0:
                raise RuntimeError(f"{self.name} login failed: {out.stderr.strip()}")
        if envc.get("force_pull_image"):
            out = subprocess.run(self.cli + ["pull", image], capture_output=True, text=True, env=cli_env)
            if out.returncode != 0:
                raise RuntimeError(f"{self.name} pull {image} failed: {out.stderr.strip()}")

    def launch(self, argv: List[str], workdir: pathlib.Path, env: Dict[str, str], cmd: Dict[str, Any]) -> TaskHandle:
        args, task_env, image = self.run_args(argv, workdir, env, cmd)
        cli_env = dict(os.environ)
        cli_env.update(task_env)
        self._prepare_image(image, env, cli_env)
        out = subprocess.run(args, capture_output=True, text=True, env=cli_env)
        if out.returncode != 0:
            raise RuntimeError(f"{self.name} run failed ({out.returncode}): {out.stderr.strip()}")
        cid = out.stdout.strip().splitlines()[-1]
        logger.info(f"{self.name}: allocation {cmd.get('allocation_id')} -> container {cid[:12]} ({image})")
        return _ContainerHandle(self, cid)

    def reattach(self) -> List[Dict[str, Any]]:
        """This agent's containers that outlived an agent restart: ``[{allocation_id, task_id, handle}]``
        (running ones are followed again; exited ones still report their exit code)."""
        fmt = "{{.ID}}\t{{.Label \"%s.allocation\"}}\t{{.Label \"%s.task\"}}" % (LABEL, LABEL)
        out = subprocess.run(self.cli + ["ps", "-a", "--filter", f"label={LABEL}.agent={self.agent_id}",
                                         "--format", fmt], capture_output=True, text=True)
        if out.returncode != 0:
            logger.warning(f"{self.name} ps failed: {out.stderr.strip()}")
            return []
        found = []
        for ln in out.stdout.splitlines():
            parts = ln.split("\t")
            if len(parts) == 3 and parts[1]:
                found.append({"allocation_id": parts[1], "task_id": parts[2], "handle": _ContainerHandle(self, parts[0])})
        return found
