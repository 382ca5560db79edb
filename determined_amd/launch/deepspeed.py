"""Launch layer for DeepSpeedTrial / ZeRO jobs (reference: ``harness/determined/launch/deepspeed.py``).

    python -m determined_amd.launch.deepspeed [TORCHRUN_OVERRIDES... --] (--trial mod:Cls | SCRIPT...)

The reference drives DeepSpeed's own runner (pdsh/ssh from the chief container, a hostfile, and
``pid_server``/``pid_client`` to notice dead workers).  Our ZeRO engine needs no DeepSpeed runtime:
every node starts ``torch.distributed.run`` for its local GPUs (one rank per GPU, RCCL over xGMI
inside the node), and every rank is wrapped in a ``pid_client`` that registers with a
``pid_server`` on the chief.  When any rank on any node dies, the chief's server SIGTERMs its
launcher, torchrun tears down the local ranks, the trial exits non-zero and the master restarts
the whole gang (``max_restarts``) -- the surviving ranks never sit in a collective waiting for a
peer that is gone.  Single-node jobs skip the supervisor (torchrun already watches its children).
"""

import json
import os
import subprocess
import sys
from typing import List

from determined_amd.launch import torch_distributed

PID_SERVER_PORT = int(os.environ.get("DET_PID_SERVER_PORT", "29411"))


def build_cmd(overrides: List[str], script: List[str], env: dict) -> List[str]:
    slots = json.loads(env.get("DET_SLOT_IDS", "[0]"))
    addrs = json.loads(env.get("DET_CONTAINER_ADDRS", '["127.0.0.1"]'))
    rank = int(env.get("DET_CONTAINER_RANK", "0"))
    nproc = len(slots) if env.get("DET_USE_GPU", "0") == "1" else int(env.get("DET_NPROC", len(slots) or 1))
    chief = addrs[0] if len(addrs) > 1 else "127.0.0.1"
    if script and script[0] == "--trial":
        script = ["-m", "determined_amd.exec.harness", script[1]]
    elif script and script[0] in ("python", "python3", sys.executable):
        script = script[1:]
    worker = [sys.executable, "-m", "determined_amd.launch.wrap_rank", "RANK", "--", sys.executable] + script
    multi = len(addrs) > 1
    if multi:
        worker = [sys.executable, "-m", "determined_amd.exec.pid_client", f"{chief}:{PID_SERVER_PORT}", "--"] + worker
    cmd = torch_distributed.create_launch_cmd(len(addrs), nproc, rank, chief, overrides) + ["--no-python"] + worker
    if multi and rank == 0:
        cmd = [sys.executable, "-m", "determined_amd.exec.pid_server", "--on-fail", "SIGTERM",
               str(PID_SERVER_PORT), str(nproc * len(addrs)), "--"] + cmd
    return cmd


def main(argv: List[str]) -> int:
    overrides, script = torch_distributed.parse_args(argv)
    if not script:
        print("usage: python -m determined_amd.launch.deepspeed [OVERRIDES --] (--trial M:C | SCRIPT...)",
              file=sys.stderr)
        return 2
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["USE_DEEPSPEED"] = "1"
    addrs = json.loads(env.get("DET_CONTAINER_ADDRS", '["127.0.0.1"]'))
    env["DET_CHIEF_IP"] = addrs[0] if len(addrs) > 1 else "127.0.0.1"
    p = subprocess.Popen(build_cmd(overrides, script, env), env=env)
    try:
        return p.wait()
    except KeyboardInterrupt:
        p.terminate()
        return p.wait()


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
