"""``python -m determined_amd.agent --master-url http://127.0.0.1:8080``"""

import argparse
import logging
import os
import shlex
import socket
import sys

from determined_amd.agent import Agent
from determined_amd.agent.backends import make_backend


def main(argv=None) -> int:
    p = argparse.ArgumentParser("determined_amd.agent")
    p.add_argument("--master-url", default=os.environ.get("DET_MASTER", "http://127.0.0.1:8080"))
    p.add_argument("--agent-id", default=None)
    p.add_argument("--slots", type=int, default=None, help="CPU slots (disables GPU detection)")
    p.add_argument("--gpus", default=None, help="comma-separated GPU ordinals to expose (default: all)")
    p.add_argument("--work-root", default=None)
    p.add_argument("--host", default=None, help="address other agents/ranks use to reach this node")
    p.add_argument("--label", default="")
    p.add_argument("--resource-pool", default=None, help="pool to join (default: the master's default compute pool)")
    p.add_argument("--backend", default="process", choices=["process", "docker", "podman", "slurm", "pbs", "kubernetes"],
                   help="where tasks run: local process groups, Docker/Podman containers, Slurm/PBS batch jobs, "
                        "or Kubernetes pods")
    p.add_argument("--default-image", default=None, help="container image when the config names none")
    p.add_argument("--gpu-slots", type=int, default=None,
                   help="GPU capacity this agent advertises (batch partitions / Kubernetes: the whole pool)")
    p.add_argument("--slots-per-node", type=int, default=8, help="GPUs per batch node / per pod")
    p.add_argument("--partition", default=None, help="Slurm partition (PBS: queue)")
    p.add_argument("--batch-args", default="", help="extra sbatch/qsub arguments (shell-quoted string)")
    p.add_argument("--k8s-api", default=None, help="Kubernetes API URL (default: in-cluster config)")
    p.add_argument("--k8s-namespace", default="default")
    p.add_argument("--k8s-image", default="determined-amd:latest")
    p.add_argument("--k8s-token-file", default=None)
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    gpus = [int(x) for x in a.gpus.split(",")] if a.gpus else None
    if a.gpu_slots is not None:
        gpus = list(range(a.gpu_slots))
    backend = None
    if a.backend in ("slurm", "pbs"):
        kw = {"slots_per_node": a.slots_per_node, "extra_args": shlex.split(a.batch_args)}
        kw["partition" if a.backend == "slurm" else "queue_name"] = a.partition
        backend = make_backend(a.backend, **kw)
    elif a.backend in ("docker", "podman"):
        kw = {"agent_id": a.agent_id or socket.gethostname()}
        if a.default_image:
            kw["default_image"] = a.default_image
        backend = make_backend(a.backend, **kw)
    elif a.backend == "kubernetes":
        token = open(a.k8s_token_file).read().strip() if a.k8s_token_file else None
        backend = make_backend("kubernetes", api_url=a.k8s_api, token=token, namespace=a.k8s_namespace,
                               image=a.k8s_image, slots_per_pod=a.slots_per_node)
    if a.backend in ("slurm", "pbs", "kubernetes") and a.slots is None and gpus is None:
        p.error(f"--backend {a.backend} fronts a whole partition: give its GPU capacity with --gpu-slots N")
    agent = Agent(a.master_url, a.agent_id, a.slots, gpus, a.work_root, a.host,
                  token=os.environ.get("DET_MASTER_TOKEN"), label=a.label, backend=backend,
                  resource_pool=a.resource_pool)
    try:
        agent.run()
    except KeyboardInterrupt:
        agent.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
