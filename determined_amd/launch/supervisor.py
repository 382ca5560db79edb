"""Worker-liveness supervision for launch layers whose workers are not our children
(reference: ``harness/determined/ipc.py:PIDServer/PIDClient``, ``exec/pid_server.py``,
``exec/pid_client.py``).

A multi-node launch starts one launcher per node; the chief also runs the user command under a
``WorkerSupervisor``.  Every worker wraps its own command in a ``WorkerClient``, which connects
to the supervisor and registers its pid.  The supervisor then waits until every registered worker
has said goodbye cleanly; if a worker's pid vanishes without a goodbye (a crashed rank, an OOM
kill, a lost node) it signals the supervised command so the whole gang comes down quickly and the
master can restart the trial, instead of the surviving ranks hanging inside an RCCL collective.

Wire protocol (one connection per worker, client -> server only):
    ``{"pid": <int>}\\n``   registration (first line)
    ``.``                  keep-alive (any number)
    ``!<exit code>\\n``     goodbye; code 0 is a graceful exit

Addresses: a path containing ``/`` is a unix socket, ``host:port`` or a bare port is TCP.
"""

import json
import logging
import os
import selectors
import signal
import socket
import subprocess
import time
from typing import Callable, Dict, List, Optional, Tuple, Union

logger = logging.getLogger("determined_amd.launch.supervisor")

Addr = Union[str, int, Tuple[str, int]]


class WorkerFailed(RuntimeError):
    """A supervised worker disappeared or exited non-zero."""


def parse_addr(addr: str) -> Addr:
    if "/" in addr:
        return addr
    host, sep, port = addr.rpartition(":")
    try:
        return (host, int(port)) if sep else int(port)
    except ValueError:
        raise ValueError(f"{addr!r} is not a unix socket path, host:port or port") from None


def parse_signal(val: str) -> Optional[signal.Signals]:
    """``WAIT`` (do nothing) or a signal name like ``SIGTERM`` / ``term``."""
    v = val.strip().upper()
    if v == "WAIT":
        return None
    if not v.startswith("SIG"):
        v = "SIG" + v
    try:
        return signal.Signals[v]
    except KeyError:
        raise ValueError(f"{val!r} is neither WAIT nor a signal name") from None


def _pid_alive(pid: int) -> bool:
    try:
        with open(f"/proc/{pid}/stat") as f:
            state = f.read().rsplit(")", 1)[1].split()[0]
        return state not in ("Z", "X", "T")
    except (FileNotFoundError, ProcessLookupError, IndexError):
        return False


def _socket_for(addr: Addr) -> socket.socket:
    return socket.socket(socket.AF_UNIX) if isinstance(addr, str) else socket.socket()


def _tcp(addr: Addr, default_host: str) -> Tuple[str, int]:
    return (default_host, addr) if isinstance(addr, int) else addr  # type: ignore[return-value]


class WorkerSupervisor:
    """Accepts ``num_workers`` registrations and watches them until all exit cleanly."""

    def __init__(self, addr: Addr, num_workers: int) -> None:
        self.addr = addr
        self.num_workers = num_workers
        self.sel: Optional[selectors.BaseSelector] = None
        self.listener: Optional[socket.socket] = None
        self.bufs: Dict[socket.socket, bytes] = {}
        self.worker_of: Dict[socket.socket, int] = {}  # connection -> worker index
        self.pids: List[int] = []  # registered pid per worker index
        self.exit_codes: Dict[int, int] = {}  # worker index -> goodbye exit code

    # ---------------------------------------------------------------- lifecycle
    def start(self) -> "WorkerSupervisor":
        self.sel = selectors.DefaultSelector()
        lst = _socket_for(self.addr)
        try:
            if isinstance(self.addr, str):
                if os.path.exists(self.addr):
                    os.unlink(self.addr)
                lst.bind(self.addr)
            else:
                lst.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
                lst.bind(_tcp(self.addr, ""))
            lst.listen(max(1, self.num_workers))
            lst.setblocking(False)
        except Exception:
            lst.close()
            raise
        self.listener = lst
        self.sel.register(lst, selectors.EVENT_READ)
        return self

    def close(self) -> None:
        for c in list(self.bufs):
            c.close()
        self.bufs.clear()
        if self.listener is not None:
            self.listener.close()
            self.listener = None
        if isinstance(self.addr, str) and os.path.exists(self.addr):
            os.unlink(self.addr)
        if self.sel is not None:
            self.sel.close()
            self.sel = None

    def __enter__(self) -> "WorkerSupervisor":
        return self.start()

    def __exit__(self, *_: object) -> None:
        self.close()

    # ---------------------------------------------------------------- events
    @property
    def all_registered(self) -> bool:
        return len(self.pids) >= self.num_workers

    @property
    def finished(self) -> bool:
        return self.all_registered and len(self.exit_codes) >= self.num_workers

    def _accept(self) -> None:
        assert self.listener is not None and self.sel is not None
        conn, _ = self.listener.accept()
        conn.setblocking(False)
        self.bufs[conn] = b""
        self.sel.register(conn, selectors.EVENT_READ)

    def _drop(self, conn: socket.socket) -> None:
        assert self.sel is not None
        self.sel.unregister(conn)
        conn.close()
        self.bufs.pop(conn, None)

    def _consume(self, conn: socket.socket) -> None:
        try:
            data = conn.recv(4096)
        except (BlockingIOError, InterruptedError):
            return
        except OSError:
            data = b""
        buf = self.bufs[conn] + data
        if conn not in self.worker_of:
            if b"\n" not in buf:
                if not data:
                    self._drop(conn)
                    raise WorkerFailed("a worker connected but never registered its pid")
                self.bufs[conn] = buf
                return
            line, buf = buf.split(b"\n", 1)
            self.worker_of[conn] = len(self.pids)
            self.pids.append(int(json.loads(line)["pid"]))
            if self.all_registered and self.listener is not None:
                assert self.sel is not None
                self.sel.unregister(self.listener)
                self.listener.close()
                self.listener = None
        w = self.worker_of[conn]
        pid = self.pids[w]
        buf = buf.replace(b".", b"")
        if b"!" in buf and b"\n" in buf.split(b"!", 1)[1]:
            code = int(buf.split(b"!", 1)[1].split(b"\n", 1)[0])
            self.exit_codes[w] = code
            self._drop(conn)
            if code != 0:
                raise WorkerFailed(f"worker pid {pid} exited with code {code}")
            return
        self.bufs[conn] = buf
        if not data:  # EOF without a goodbye
            self._drop(conn)
            raise WorkerFailed(f"worker pid {pid} disconnected without exiting cleanly")

    def check_pids(self) -> None:
        for w, pid in enumerate(self.pids):
            if w not in self.exit_codes and not _pid_alive(pid):
                raise WorkerFailed(f"worker pid {pid} died")

    def run(self, health_check: Optional[Callable[[], None]] = None, poll_s: float = 0.5) -> None:
        """Block until every worker registered and exited 0; raise WorkerFailed otherwise."""
        assert self.sel is not None, "start() first"
        while not self.finished:
            for key, _ in self.sel.select(timeout=poll_s):
                if key.fileobj is self.listener:
                    self._accept()
                else:
                    self._consume(key.fileobj)  # type: ignore[arg-type]
            self.check_pids()
            if health_check is not None:
                health_check()

    def run_subprocess(self, cmd: List[str], on_fail: Optional[signal.Signals] = signal.SIGTERM,
                       on_exit: Optional[signal.Signals] = None, grace_s: float = 3.0,
                       signal_group: bool = False) -> int:
        """Run ``cmd`` while supervising; on a worker failure signal ``cmd`` with ``on_fail``."""
        p = subprocess.Popen(cmd, start_new_session=signal_group)

        class _Exited(Exception):
            pass

        def health() -> None:
            if p.poll() is not None:
                raise _Exited()

        def send(sig: signal.Signals) -> None:
            try:
                if signal_group:
                    os.killpg(p.pid, sig)
                else:
                    p.send_signal(sig)
            except ProcessLookupError:
                pass

        def finish(sig: Optional[signal.Signals], default_code: int) -> int:
            if sig is not None:
                time.sleep(grace_s)
                send(sig)
                try:
                    return p.wait(timeout=10) or default_code
                except subprocess.TimeoutExpired:
                    logger.error("supervised command ignored %s; killing it", sig.name)
                    send(signal.SIGKILL)
            return p.wait() or default_code

        old = {s: signal.signal(s, lambda n, _f: send(signal.Signals(n))) for s in (signal.SIGTERM, signal.SIGINT)}
        try:
            try:
                self.run(health)
            except _Exited:
                return p.returncode if p.returncode else (0 if self.finished else 77)
            except WorkerFailed as e:
                logger.error("%s; signalling the launch", e)
                return finish(on_fail, 78)
            return finish(on_exit, 0) if on_exit is not None else p.wait()
        finally:
            for s, h in old.items():
                signal.signal(s, h)


class WorkerClient:
    """Registers this process with a WorkerSupervisor; ``close(code)`` says goodbye."""

    def __init__(self, addr: Addr, connect_timeout_s: float = 60.0) -> None:
        self.addr = addr
        self.connect_timeout_s = connect_timeout_s
        self.sock: Optional[socket.socket] = None

    def start(self) -> "WorkerClient":
        deadline = time.monotonic() + self.connect_timeout_s
        while True:
            s = _socket_for(self.addr)
            try:
                s.connect(self.addr if isinstance(self.addr, str) else _tcp(self.addr, "127.0.0.1"))
                break
            except (ConnectionRefusedError, FileNotFoundError):
                s.close()
                if time.monotonic() > deadline:
                    raise
                time.sleep(0.1)
        s.sendall(json.dumps({"pid": os.getpid()}).encode() + b"\n")
        self.sock = s
        return self

    def keep_alive(self) -> None:
        assert self.sock is not None
        self.sock.sendall(b".")

    def close(self, exit_code: int = 0) -> None:
        if self.sock is None:
            return
        try:
            self.sock.sendall(b"!%d\n" % exit_code)
        except OSError:
            pass
        self.sock.close()
        self.sock = None

    def __enter__(self) -> "WorkerClient":
        return self.start()

    def __exit__(self, etype: Optional[type], exc: Optional[BaseException], _tb: object) -> None:
        if etype is None:
            code = 0
        elif isinstance(exc, SystemExit):
            code = exc.code if isinstance(exc.code, int) else (0 if exc.code is None else 1)
        else:
            code = 1
        self.close(code)

    def run_subprocess(self, cmd: List[str], keepalive_s: float = 30.0) -> int:
        p = subprocess.Popen(cmd)
        old = {s: signal.signal(s, lambda n, _f: p.send_signal(n)) for s in (signal.SIGTERM, signal.SIGINT)}
        try:
            while True:
                try:
                    return p.wait(timeout=keepalive_s)
                except subprocess.TimeoutExpired:
                    self.keep_alive()
        finally:
            for s, h in old.items():
                signal.signal(s, h)
