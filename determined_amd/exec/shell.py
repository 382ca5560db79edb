"""Shell task (reference: ``det shell``, which runs sshd inside the task container).

Our tasks are process groups on the agent host, so a shell needs no server of its own: this task
only *holds the allocation* (the slots stay reserved for the user) and publishes where it runs
and which devices it owns.  ``det shell open`` then starts an interactive ``bash`` on that host
with the allocation's environment (``HIP_VISIBLE_DEVICES`` = the allocated GPUs, ``DET_*``):
directly when the agent is local, otherwise through the host's own ``ssh`` (the command is what
``det shell show-ssh-command`` prints).  No network listener is opened by the task.  It ends on
``det shell kill`` or after ``--idle-timeout`` seconds.
"""

import argparse
import json
import os
import signal
import sys
import time
from typing import List


def environment() -> dict:
    """The variables a shell in this allocation should see."""
    keep = ("HIP_VISIBLE_DEVICES", "DET_MASTER", "DET_TASK_ID", "DET_ALLOCATION_ID", "DET_SLOT_IDS",
            "DET_AGENT_ID", "DET_CONTAINER_ADDRS", "DET_CONTAINER_RANK", "DET_USE_GPU", "DET_CPU_SLOTS",
            "HSA_ENABLE_IPC_MODE_LEGACY")
    return {k: os.environ[k] for k in keep if k in os.environ}


def publish() -> None:
    master, task = os.environ.get("DET_MASTER"), os.environ.get("DET_TASK_ID")
    if not (master and task):
        return
    from determined_amd.common.api import Session

    Session(master, token=os.environ.get("DET_SESSION_TOKEN") or None).post(
        f"/api/v1/tasks/{task}/proxy", {"host": os.environ.get("DET_AGENT_HOST", "127.0.0.1"), "port": None,
                                        "cwd": os.getcwd(), "env": environment()})


def main(argv: List[str]) -> int:
    ap = argparse.ArgumentParser(prog="shell")
    ap.add_argument("--idle-timeout", type=float, default=0.0, help="release the slots after N seconds (0: never)")
    a = ap.parse_args(argv)
    stop = {"now": False}
    signal.signal(signal.SIGTERM, lambda *_: stop.update(now=True))
    publish()
    print(f"shell allocation ready: {json.dumps(environment())}", flush=True)
    t0 = time.monotonic()
    while not stop["now"]:
        time.sleep(0.5)
        if a.idle_timeout and time.monotonic() - t0 > a.idle_timeout:
            break
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
