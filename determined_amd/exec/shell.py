"""Shell task (reference: ``det shell``, which runs sshd inside the task container and tunnels ssh
through the master: ``harness/determined/cli/shell.py``, ``cli/tunnel.py``).

Here the task runs a small PTY server instead of sshd: it listens on a free TCP port of the agent's
own address (the one the master reaches the node on; loopback for a local agent), publishes
``{host, port, shell_key}`` to the master (``POST /api/v1/tasks/<id>/proxy``), and serves shells
and one-off commands with the allocation's environment (``HIP_VISIBLE_DEVICES`` = the allocated
GPUs, ``DET_*``).  Clients never connect to it directly: ``det shell open`` asks the master for a
tunnel (``/proxy/<task>/_tunnel`` with an ``Upgrade: damd-tunnel`` header); the master checks the
user may use the task, opens the TCP connection, sends the shell key as the first line and then
relays bytes both ways.  So a shell works on any agent the master can reach, with no ssh access to
the node.

Wire format after the key line (both directions framed as ``type(1) length(4, big endian) payload``):

* client -> server: ``c`` (first frame) JSON ``{"argv": [...] | null, "tty": bool, "rows", "cols"}``;
  ``d`` stdin bytes; ``r`` window size (rows, cols as two big-endian u16); ``e`` stdin EOF.
* server -> client: ``o`` output bytes; ``x`` exit status (big-endian i32), then close.

The task ends on ``det shell kill`` or after ``--idle-timeout`` seconds without a connected client.
"""

import argparse
import fcntl
import hmac
import json
import os
import secrets
import select
import signal
import socket
import struct
import subprocess
import sys
import termios
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

MAGIC = b"DAMD-SHELL "


def environment() -> dict:
    """The variables a shell in this allocation should see."""
    keep = ("HIP_VISIBLE_DEVICES", "DET_MASTER", "DET_TASK_ID", "DET_ALLOCATION_ID", "DET_SLOT_IDS",
            "DET_AGENT_ID", "DET_CONTAINER_ADDRS", "DET_CONTAINER_RANK", "DET_USE_GPU", "DET_CPU_SLOTS",
            "HSA_ENABLE_IPC_MODE_LEGACY")
    return {k: os.environ[k] for k in keep if k in os.environ}


# ------------------------------------------------------------------------------------------ framing
def send_frame(sock: socket.socket, kind: bytes, payload: bytes = b"") -> None:
    sock.sendall(kind + struct.pack(">I", len(payload)) + payload)


def _recv_exact(sock: socket.socket, n: int) -> Optional[bytes]:
    buf = b""
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            return None
        buf += chunk
    return buf


def recv_frame(sock: socket.socket) -> Optional[Tuple[bytes, bytes]]:
    head = _recv_exact(sock, 5)
    if head is None:
        return None
    (n,) = struct.unpack(">I", head[1:])
    payload = _recv_exact(sock, n) if n else b""
    if payload is None:
        return None
    return head[:1], payload


# ------------------------------------------------------------------------------------------ server
def _set_winsize(fd: int, rows: int, cols: int) -> None:
    fcntl.ioctl(fd, termios.TIOCSWINSZ, struct.pack("HHHH", rows, cols, 0, 0))


class ShellServer:
    def __init__(self, key: str, host: Optional[str] = None, cwd: Optional[str] = None) -> None:
        # only the address the master reaches this node on (loopback for a local agent): the
        # server never listens on every interface
        host = host or os.environ.get("DET_AGENT_HOST") or "127.0.0.1"
        self.key = key.encode()
        self.cwd = cwd or os.getcwd()
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((host, 0))
        self.sock.listen(16)
        self.port = self.sock.getsockname()[1]
        self.active = 0
        self.last_activity = time.monotonic()
        self._lock = threading.Lock()

    def serve_forever(self) -> None:
        while True:
            try:
                conn, _ = self.sock.accept()
            except OSError:
                return
            threading.Thread(target=self._session, args=(conn,), daemon=True).start()

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass

    def _auth(self, conn: socket.socket) -> bool:
        line = b""
        conn.settimeout(10)
        while not line.endswith(b"\n") and len(line) < 256:
            ch = conn.recv(1)
            if not ch:
                return False
            line += ch
        conn.settimeout(None)
        return line.startswith(MAGIC) and hmac.compare_digest(line[len(MAGIC):].strip(), self.key)

    def _session(self, conn: socket.socket) -> None:
        with self._lock:
            self.active += 1
        try:
            if not self._auth(conn):
                conn.close()
                return
            first = recv_frame(conn)
            if first is None or first[0] != b"c":
                conn.close()
                return
            req = json.loads(first[1] or b"{}")
            argv = req.get("argv") or [os.environ.get("SHELL") or "/bin/bash", "-l"]
            code = self._run_tty(conn, argv, req) if req.get("tty") else self._run_pipe(conn, argv)
            send_frame(conn, b"x", struct.pack(">i", code))
        except OSError:
            pass
        finally:
            with self._lock:
                self.active -= 1
                self.last_activity = time.monotonic()
            try:
                conn.close()
            except OSError:
                pass

    def _run_tty(self, conn: socket.socket, argv: List[str], req: Dict[str, Any]) -> int:
        master_fd, slave_fd = os.openpty()
        _set_winsize(slave_fd, int(req.get("rows") or 24), int(req.get("cols") or 80))
        env = dict(os.environ, TERM=req.get("term") or os.environ.get("TERM", "xterm-256color"))
        proc = subprocess.Popen(argv, stdin=slave_fd, stdout=slave_fd, stderr=slave_fd, cwd=self.cwd, env=env,
                                start_new_session=True, close_fds=True,
                                preexec_fn=lambda: fcntl.ioctl(0, termios.TIOCSCTTY, 0))
        os.close(slave_fd)
        try:
            self._relay(conn, master_fd, master_fd, proc, tty=True)
        finally:
            os.close(master_fd)
        return proc.wait()

    def _run_pipe(self, conn: socket.socket, argv: List[str]) -> int:
        proc = subprocess.Popen(argv, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                cwd=self.cwd, start_new_session=True)
        assert proc.stdin is not None and proc.stdout is not None
        self._relay(conn, proc.stdout.fileno(), proc.stdin.fileno(), proc, tty=False)
        return proc.wait()

    def _relay(self, conn: socket.socket, out_fd: int, in_fd: int, proc: subprocess.Popen, tty: bool) -> None:
        stdin_open = True
        while True:
            r, _, _ = select.select([conn, out_fd], [], [], 0.5)
            if out_fd in r:
                try:
                    data = os.read(out_fd, 65536)
                except OSError:  # pty closed: the shell exited
                    data = b""
                if not data:
                    return
                send_frame(conn, b"o", data)
            if conn in r:
                fr = recv_frame(conn)
                if fr is None:  # client went away: hang up the shell
                    try:
                        os.killpg(proc.pid, signal.SIGHUP)
                    except ProcessLookupError:
                        pass
                    return
                kind, payload = fr
                if kind == b"d" and stdin_open:
                    os.write(in_fd, payload)
                elif kind == b"r" and tty and len(payload) == 4:
                    rows, cols = struct.unpack(">HH", payload)
                    _set_winsize(out_fd, rows, cols)
                    try:
                        os.killpg(proc.pid, signal.SIGWINCH)
                    except ProcessLookupError:
                        pass
                elif kind == b"e" and stdin_open:
                    if tty:
                        os.write(in_fd, b"\x04")
                    elif proc.stdin is not None:
                        proc.stdin.close()  # the pipe's own object closes its fd (no double close)
                    stdin_open = False
            if proc.poll() is not None and not tty:
                rest = b""
                while True:  # drain what the command wrote before exiting
                    rr, _, _ = select.select([out_fd], [], [], 0.1)
                    if not rr:
                        break
                    chunk = os.read(out_fd, 65536)
                    if not chunk:
                        break
                    rest += chunk
                if rest:
                    send_frame(conn, b"o", rest)
                return


def publish(port: int, key: str) -> None:
    master, task = os.environ.get("DET_MASTER"), os.environ.get("DET_TASK_ID")
    if not (master and task):
        return
    from determined_amd.common.api import Session

    Session(master, token=os.environ.get("DET_SESSION_TOKEN") or None).post(
        f"/api/v1/tasks/{task}/proxy", {"host": os.environ.get("DET_AGENT_HOST", "127.0.0.1"), "port": port,
                                        "cwd": os.getcwd(), "env": environment(), "tunnel": True,
                                        "shell_key": key})


def main(argv: List[str]) -> int:
    ap = argparse.ArgumentParser(prog="shell")
    ap.add_argument("--idle-timeout", type=float, default=0.0,
                    help="release the slots after N seconds without a connected client (0: never)")
    a = ap.parse_args(argv)
    stop = {"now": False}
    signal.signal(signal.SIGTERM, lambda *_: stop.update(now=True))
    key = secrets.token_hex(24)
    server = ShellServer(key)
    threading.Thread(target=server.serve_forever, daemon=True).start()
    publish(server.port, key)
    print(f"shell server ready on port {server.port}: {json.dumps(environment())}", flush=True)
    while not stop["now"]:
        time.sleep(0.5)
        if a.idle_timeout and server.active == 0 and time.monotonic() - server.last_activity > a.idle_timeout:
            break
    server.close()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
