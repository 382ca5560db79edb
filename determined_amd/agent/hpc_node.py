"""Per-node entry of a task run by a batch scheduler or on Kubernetes (see ``agent/backends.py``).

``python -m determined_amd.agent.hpc_node {slurm|pbs|kubernetes} [--env-file F] -- ARGV...``

The master's ``DET_CONTAINER_RANK`` / ``DET_CONTAINER_ADDRS`` describe agent-launched gangs;
inside a batch job or a set of pods they are only known at run time, so this wrapper derives
them -- Slurm: ``SLURM_NODEID`` + the expanded ``SLURM_JOB_NODELIST``; PBS: this host's position
in ``$PBS_NODEFILE``; Kubernetes: the pod's rank (set in its manifest) + the pod IPs exchanged
through the master's allocation all-gather -- then runs ARGV (the torchrun launcher) as a child
process and exits with its status.  It never touches the GPU itself.
"""

import argparse
import json
import os
import re
import socket
import subprocess
import sys
from typing import Dict, List, Tuple


def expand_hostlist(spec: str) -> List[str]:
    """Slurm hostlist syntax: ``gpu[01-03,07],login1`` -> ``[gpu01, gpu02, gpu03, gpu07, login1]``."""
    out: List[str] = []
    for part in re.findall(r"[^,\[]+(?:\[[^\]]*\])?[^,]*", spec):
        m = re.match(r"^(.*?)\[([^\]]*)\](.*)$", part)
        if not m:
            if part:
                out.append(part)
            continue
        pre, body, post = m.groups()
        for rng in body.split(","):
            if "-" in rng:
                lo, hi = rng.split("-", 1)
                width = len(lo)
                out += [f"{pre}{i:0{width}d}{post}" for i in range(int(lo), int(hi) + 1)]
            else:
                out.append(f"{pre}{rng}{post}")
    return out


def _resolve(host: str) -> str:
    try:
        return socket.gethostbyname(host)
    except OSError:
        return host


def slurm_layout(env: Dict[str, str]) -> Tuple[int, List[str]]:
    hosts = expand_hostlist(env.get("SLURM_JOB_NODELIST") or env.get("SLURM_NODELIST") or socket.gethostname())
    return int(env.get("SLURM_NODEID", "0")), [_resolve(h) for h in hosts]


def pbs_layout(env: Dict[str, str]) -> Tuple[int, List[str]]:
    hosts: List[str] = []
    path = env.get("PBS_NODEFILE")
    if path and os.path.exists(path):
        for line in open(path).read().split():
            if line not in hosts:
                hosts.append(line)
    me = socket.gethostname()
    short = lambda h: h.split(".")[0]  # noqa: E731
    if not hosts:
        return 0, [_resolve(me)]
    rank = next((i for i, h in enumerate(hosts) if short(h) == short(me)), 0)
    return rank, [_resolve(h) for h in hosts]


def kubernetes_layout(env: Dict[str, str]) -> Tuple[int, List[str]]:
    rank = int(env.get("DET_CONTAINER_RANK", "0"))
    npods = int(env.get("DET_K8S_NUM_PODS", "1"))
    me = env.get("DET_POD_IP") or _resolve(socket.gethostname())
    if npods <= 1:
        return rank, [me]
    from determined_amd.common.api import Session

    sess = Session(env["DET_MASTER"], token=env.get("DET_SESSION_TOKEN") or None)
    # one uuid per call: Session's retries re-send the same body, so a post whose response was lost
    # re-fetches the finished round; a restarted pod (new address) joins a new round
    import uuid

    got = sess.post(f"/api/v1/allocations/{env['DET_ALLOCATION_ID']}/all_gather",
                    {"request_uuid": f"rank-{rank}-{uuid.uuid4().hex}", "num_peers": npods, "rank": rank, "data": me,
                     "timeout_seconds": 1800}, timeout=1900)
    return rank, list(got["data"])


def main(argv: List[str]) -> int:
    if "--" not in argv:
        print(__doc__, file=sys.stderr)
        return 2
    i = argv.index("--")
    ap = argparse.ArgumentParser(prog="hpc_node")
    ap.add_argument("kind", choices=["slurm", "pbs", "kubernetes"])
    ap.add_argument("--env-file", default=None)
    a = ap.parse_args(argv[:i])
    cmd = argv[i + 1:]
    env = dict(os.environ)
    if a.env_file:
        with open(a.env_file) as f:
            env.update({k: str(v) for k, v in json.load(f).items()})
    rank, addrs = {"slurm": slurm_layout, "pbs": pbs_layout, "kubernetes": kubernetes_layout}[a.kind](env)
    env["DET_CONTAINER_RANK"] = str(rank)
    env["DET_CONTAINER_ADDRS"] = json.dumps(addrs)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if a.kind == "kubernetes" and env.get("DET_EXPERIMENT_ID"):
        # pods do not share the agent's work directory: fetch the model definition from the master
        from determined_amd.exec.prep_container import main as prep

        saved = dict(os.environ)
        os.environ.update(env)
        try:
            prep(["--download-context"])
        finally:
            os.environ.clear()
            os.environ.update(saved)
        env["PYTHONPATH"] = os.pathsep.join([os.getcwd()] + [p for p in [env.get("PYTHONPATH")] if p])
    p = subprocess.Popen(cmd, env=env)
    try:
        return p.wait()
    except KeyboardInterrupt:
        p.terminate()
        return p.wait()


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
