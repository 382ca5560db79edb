"""``python -m determined_amd.exec.pid_server [-x SIG] [-e SIG] ADDR NUM_WORKERS CMD...``
(reference: ``harness/determined/exec/pid_server.py``).

Runs CMD (the launcher) while ``NUM_WORKERS`` workers register over ADDR (see
``launch/supervisor.py``).  A worker that dies without a clean exit makes the server send the
``--on-fail`` signal (default SIGTERM) to CMD; ``--on-exit`` (default WAIT) is sent once every
worker exited cleanly.
"""

import argparse
import logging
import sys
from typing import List

from determined_amd.launch.supervisor import WorkerSupervisor, parse_addr, parse_signal


def main(argv: List[str]) -> int:
    ap = argparse.ArgumentParser(prog="pid_server")
    ap.add_argument("-x", "--on-fail", default="SIGTERM")
    ap.add_argument("-e", "--on-exit", default="WAIT")
    ap.add_argument("--grace-period", type=float, default=3.0)
    ap.add_argument("--signal-children", action="store_true", help="signal CMD's whole process group")
    ap.add_argument("addr")
    ap.add_argument("num_workers", type=int)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if not a.cmd:
        ap.error("missing CMD")
    cmd = a.cmd[1:] if a.cmd[0] == "--" else a.cmd
    logging.basicConfig(level=logging.INFO)
    with WorkerSupervisor(parse_addr(a.addr), a.num_workers) as sup:
        return sup.run_subprocess(cmd, on_fail=parse_signal(a.on_fail), on_exit=parse_signal(a.on_exit),
                                  grace_s=a.grace_period, signal_group=a.signal_children)


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
