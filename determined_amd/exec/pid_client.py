"""``python -m determined_amd.exec.pid_client ADDR -- CMD...`` (reference:
``harness/determined/exec/pid_client.py``): register with a pid_server, run CMD, report its exit
code as the goodbye."""

import sys
from typing import List

from determined_amd.launch.supervisor import WorkerClient, parse_addr


def main(argv: List[str]) -> int:
    if len(argv) < 2:
        print("usage: pid_client ADDR [--] CMD...", file=sys.stderr)
        return 2
    addr, cmd = argv[0], argv[1:]
    if cmd and cmd[0] == "--":
        cmd = cmd[1:]
    client = WorkerClient(parse_addr(addr)).start()
    code = 1
    try:
        code = client.run_subprocess(cmd)
    finally:
        client.close(code)
    return code


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
