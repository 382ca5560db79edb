"""Client side of ``det shell open``: a shell (or one command) in a shell task through the master's
tunnel (reference: ``harness/determined/cli/tunnel.py`` + ssh; here the master relays the task's
PTY server, see ``determined_amd/exec/shell.py`` for the wire format)."""

import json
import os
import select
import signal
import socket
import ssl
import struct
import sys
import threading
import urllib.parse
from typing import BinaryIO, List, Optional

from determined_amd.exec.shell import recv_frame, send_frame


def open_tunnel(master_url: str, task_id: str, token: Optional[str] = None, timeout: float = 30.0) -> socket.socket:
    """An upgraded connection to the task's shell server through the master."""
    u = urllib.parse.urlparse(master_url if "://" in master_url else "http://" + master_url)
    port = u.port or (443 if u.scheme == "https" else 80)
    sock = socket.create_connection((u.hostname or "127.0.0.1", port), timeout=timeout)
    if u.scheme == "https":
        sock = ssl.create_default_context().wrap_socket(sock, server_hostname=u.hostname)
    lines = [f"GET /proxy/{task_id}/_tunnel HTTP/1.1", f"Host: {u.netloc}", "Upgrade: damd-tunnel",
             "Connection: Upgrade", "Content-Length: 0"]
    if token:
        lines.append(f"Authorization: Bearer {token}")
    sock.sendall(("\r\n".join(lines) + "\r\n\r\n").encode())
    head = b""
    while b"\r\n\r\n" not in head:
        chunk = sock.recv(1)
        if not chunk:
            raise ConnectionError("master closed the tunnel request")
        head += chunk
    status = head.split(b"\r\n", 1)[0].decode(errors="replace")
    if " 101 " not in status + " ":
        body = b""
        try:
            sock.settimeout(2)
            body = sock.recv(4096)
        except OSError:
            pass
        raise ConnectionError(f"tunnel refused: {status} {body.decode(errors='replace').strip()}")
    sock.settimeout(None)
    return sock


def run(master_url: str, task_id: str, argv: Optional[List[str]] = None, token: Optional[str] = None,
        stdin: Optional[BinaryIO] = None, stdout: Optional[BinaryIO] = None, tty: Optional[bool] = None) -> int:
    """Run ``argv`` (default: a login shell) in the task; relays stdin / stdout; returns the exit
    status.  With a terminal on stdin the session is interactive (raw mode, window-size updates)."""
    stdin = stdin if stdin is not None else sys.stdin.buffer
    stdout = stdout if stdout is not None else sys.stdout.buffer
    in_fd = stdin.fileno() if hasattr(stdin, "fileno") else None
    if tty is None:
        tty = in_fd is not None and os.isatty(in_fd)
    sock = open_tunnel(master_url, task_id, token)
    rows, cols = 24, 80
    if tty:
        try:
            cols, rows = os.get_terminal_size(in_fd)
        except OSError:
            pass
    send_frame(sock, b"c", json.dumps({"argv": argv or None, "tty": bool(tty), "rows": rows, "cols": cols,
                                       "term": os.environ.get("TERM")}).encode())
    saved = None
    if tty:
        import termios
        import tty as ttymod

        saved = termios.tcgetattr(in_fd)
        ttymod.setraw(in_fd)

        def winch(*_):
            try:
                c, r = os.get_terminal_size(in_fd)
                send_frame(sock, b"r", struct.pack(">HH", r, c))
            except OSError:
                pass

        signal.signal(signal.SIGWINCH, winch)
    done = threading.Event()

    def pump_stdin() -> None:
        try:
            while not done.is_set():
                if in_fd is not None:
                    r, _, _ = select.select([in_fd], [], [], 0.2)
                    if not r:
                        continue
                    data = os.read(in_fd, 65536)
                else:
                    data = stdin.read(65536)
                if not data:
                    send_frame(sock, b"e")
                    return
                send_frame(sock, b"d", data)
        except OSError:
            return

    threading.Thread(target=pump_stdin, daemon=True).start()
    code = 255
    try:
        while True:
            fr = recv_frame(sock)
            if fr is None:
                break
            kind, payload = fr
            if kind == b"o":
                stdout.write(payload)
                stdout.flush()
            elif kind == b"x":
                (code,) = struct.unpack(">i", payload)
                break
    finally:
        done.set()
        if saved is not None:
            import termios

            termios.tcsetattr(in_fd, termios.TCSADRAIN, saved)
        sock.close()
    return code
