"""Launch a task on every slot with ``torch.distributed.run`` (one process per GPU, RCCL over xGMI)
(reference: ``harness/determined/launch/torch_distributed.py``; replaces the Horovod launcher too).

    python -m determined_amd.launch.torch_distributed [TORCHRUN_OVERRIDES... --] (--trial mod:Cls | SCRIPT...)

Every rank's output is prefixed ``[rank=N]`` by ``wrap_rank`` so the agent can attribute logs.
``--max-restarts 0``: if one rank dies torchrun tears the others down and the master decides
whether to restart the whole trial (``max_restarts``).  ``HSA_ENABLE_IPC_MODE_LEGACY=0`` is kept in
the environment: the host driver only supports dmabuf IPC for RCCL peer buffers.
"""

import json
import os
import subprocess
import sys
from typing import List, Tuple

C10D_PORT = int(os.environ.get("C10D_PORT", "29400"))


def create_launch_cmd(num_nodes: int, proc_per_node: int, node_rank: int, master_addr: str,
                      override_args: List[str]) -> List[str]:
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", str(num_nodes), "--nproc-per-node",
            str(proc_per_node), "--node-rank", str(node_rank), "--max-restarts", "0", "--master-addr", master_addr,
            "--master-port", str(C10D_PORT), *override_args]


def parse_args(args: List[str]) -> Tuple[List[str], List[str]]:
    if "--" in args:
        i = args.index("--")
        return args[:i], args[i + 1:]
    return [], args


def main(argv: List[str]) -> int:
    overrides, script = parse_args(argv)
    if not script:
        print("usage: python -m determined_amd.launch.torch_distributed [OVERRIDES --] (--trial M:C | SCRIPT...)",
              file=sys.stderr)
        return 2
    if script[0] == "--trial":
        script = ["-m", "determined_amd.exec.harness", script[1]]
    elif script[0] in ("python", "python3", sys.executable):
        script = script[1:]
    slots = json.loads(os.environ.get("DET_SLOT_IDS", "[0]"))
    addrs = json.loads(os.environ.get("DET_CONTAINER_ADDRS", '["127.0.0.1"]'))
    rank = int(os.environ.get("DET_CONTAINER_RANK", "0"))
    nproc = len(slots) if os.environ.get("DET_USE_GPU", "0") == "1" else int(os.environ.get("DET_NPROC", len(slots) or 1))
    chief = addrs[0] if len(addrs) > 1 else "127.0.0.1"
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["DET_CHIEF_IP"] = chief
    env["USE_TORCH_DISTRIBUTED"] = "True"
    cmd = create_launch_cmd(len(addrs), nproc, rank, chief, overrides) + \
        ["--no-python", sys.executable, "-m", "determined_amd.launch.wrap_rank", "RANK", "--",
         sys.executable] + script
    p = subprocess.Popen(cmd, env=env)
    try:
        return p.wait()
    except KeyboardInterrupt:
        p.terminate()
        return p.wait()


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
