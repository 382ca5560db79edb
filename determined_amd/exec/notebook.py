"""Notebook task (reference: ``det notebook``, a JupyterLab server in the task container).

Runs ``jupyter lab`` bound to the agent's loopback interface with a per-task token and
registers the address with the master.  JupyterLab is not installed in this image: the task
then exits at once with a clear message (which ``det notebook start`` shows) instead of hanging.
"""

import os
import shutil
import socket
import subprocess
import sys
from typing import List


def jupyter_available() -> bool:
    if shutil.which("jupyter") is None:
        return False
    try:
        import jupyterlab  # noqa: F401
    except ImportError:
        return False
    return True


def main(argv: List[str]) -> int:
    if not jupyter_available():
        print("notebook task: JupyterLab is not installed in this environment "
              "(install jupyterlab into the agent's Python to enable notebooks)", file=sys.stderr, flush=True)
        return 3
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    token = os.environ.get("DET_NOTEBOOK_TOKEN", "")
    from determined_amd.exec.tensorboard import register_address

    p = subprocess.Popen(["jupyter", "lab", "--ip", "127.0.0.1", "--port", str(port), "--no-browser",
                          f"--ServerApp.token={token}", "--ServerApp.root_dir", os.getcwd()] + argv)
    register_address(port)
    return p.wait()


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
