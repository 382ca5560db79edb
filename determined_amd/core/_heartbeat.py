"""Trial-state reporting for unmanaged (detached) trials (reference ``core/_heartbeat.py``).

A managed trial's state belongs to the master (it launched the process and sees it exit).  An
unmanaged trial runs wherever the user started it, so the chief reports it instead:

* on ``core.init()`` enter: the trial is RUNNING;
* every ``interval`` seconds: a heartbeat, which the master records as the trial's last activity --
  a trial whose heartbeats stop (the process was killed, the node died) is marked ERROR by the master
  once ``unmanaged_timeout_s`` passes (``Master._reap_unmanaged``);
* on exit: COMPLETED, or ERROR when the context exits with an exception, an uncaught exception reached
  ``sys.excepthook``, or ``sys.exit`` was called with a non-zero code.
"""

import logging
import sys
import threading
import types
from typing import Any, Optional

logger = logging.getLogger("determined_amd.core")


class _ExitHook:
    """Remembers an uncaught exception / a non-zero ``sys.exit`` while installed."""

    def __init__(self) -> None:
        self.exit_code: Any = None
        self.exception: Optional[BaseException] = None
        self._orig_exit = None
        self._orig_excepthook = None

    def install(self) -> None:
        self._orig_exit, self._orig_excepthook = sys.exit, sys.excepthook
        sys.exit = self._exit  # type: ignore[assignment]
        sys.excepthook = self._excepthook

    def uninstall(self) -> None:
        if self._orig_exit is not None:
            if sys.exit == self._exit:  # type: ignore[comparison-overlap]
                sys.exit = self._orig_exit  # type: ignore[assignment]
            if sys.excepthook == self._excepthook:
                sys.excepthook = self._orig_excepthook  # type: ignore[assignment]

    def _exit(self, code: Any = 0) -> None:
        self.exit_code = code
        self._orig_exit(code)  # type: ignore[misc]

    def _excepthook(self, exc_type: Any, exc: BaseException, tb: Any) -> None:
        self.exception = exc
        self._orig_excepthook(exc_type, exc, tb)  # type: ignore[misc]


class UnmanagedTrialHeartbeat:
    def __init__(self, session: Any, trial_id: int, interval: float = 60.0) -> None:
        self._session = session
        self._trial_id = trial_id
        self._interval = interval
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._hook = _ExitHook()
        self.final_state: Optional[str] = None
        self.requested_state: Optional[str] = None  # core_v2.close(state=...): the state of a clean exit

    def _patch(self, body: Any) -> None:
        self._session.patch(f"/api/v1/trials/{self._trial_id}", body)

    def _run(self) -> None:
        while not self._stop.wait(self._interval):
            try:
                self._patch({"heartbeat": True})
            except Exception as e:  # the master is restarting / unreachable: keep trying
                logger.warning(f"unmanaged trial heartbeat failed (retrying): {e}")

    def start(self) -> "UnmanagedTrialHeartbeat":
        self._patch({"state": "RUNNING"})
        self._thread = threading.Thread(target=self._run, name="det-heartbeat", daemon=True)
        self._thread.start()
        self._hook.install()
        return self

    def close(self, exc_type: Optional[type] = None, exc_val: Optional[BaseException] = None,
              exc_tb: Optional[types.TracebackType] = None) -> None:
        if self.final_state is not None:
            return
        self._stop.set()
        self._hook.uninstall()
        failed = exc_type is not None or self._hook.exception is not None or \
            (self._hook.exit_code not in (None, 0))
        self.final_state = "ERROR" if failed else (self.requested_state or "COMPLETED")
        if failed:
            logger.error(f"unmanaged trial {self._trial_id} ends in ERROR: "
                         f"{exc_val or self._hook.exception or f'exit code {self._hook.exit_code}'}")
        try:
            self._patch({"state": self.final_state})
        except Exception as e:
            logger.warning(f"could not report the final state of trial {self._trial_id}: {e}")
