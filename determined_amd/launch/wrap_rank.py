"""Prefix every output line of a rank with ``[rank=N] `` (reference: ``harness/determined/launch/wrap_rank.py``).

    python -m determined_amd.launch.wrap_rank RANK -- CMD...

``RANK`` names an environment variable (set by torchrun) or is a literal integer.  The child is
started as a subprocess (never exec'd) and its exit code is returned.
"""

import os
import subprocess
import sys
import threading
from typing import IO, List


def _pump(src: IO[bytes], dst: IO[bytes], prefix: bytes) -> None:
    for line in iter(src.readline, b""):
        dst.write(prefix + line)
        dst.flush()


def main(argv: List[str]) -> int:
    if len(argv) < 3 or argv[1] != "--":
        print("usage: wrap_rank RANK -- CMD...", file=sys.stderr)
        return 2
    rank_spec, cmd = argv[0], argv[2:]
    rank = os.environ.get(rank_spec, rank_spec)
    prefix = f"[rank={rank}] ".encode()
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    ts = [threading.Thread(target=_pump, args=(p.stdout, sys.stdout.buffer, prefix), daemon=True),
          threading.Thread(target=_pump, args=(p.stderr, sys.stderr.buffer, prefix), daemon=True)]
    for t in ts:
        t.start()
    code = p.wait()
    for t in ts:
        t.join(timeout=5)
    return code


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
