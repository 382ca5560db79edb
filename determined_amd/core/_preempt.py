"""PreemptContext (reference: ``harness/determined/core/_preempt.py``).

A watcher thread long-polls the master's preemption signal for this allocation; the chief's
answer is broadcast to workers (``WorkersAskChief``) so every rank stops at the same step.
"""

import enum
import logging
import threading
from typing import Any, Optional

logger = logging.getLogger("determined_amd.core")


class _PreemptionWatcher(threading.Thread):
    def __init__(self, session: Any, allocation_id: str, longpoll_s: int = 60) -> None:
        super().__init__(daemon=True, name="preemption-watcher")
        self._session = session
        self._allocation_id = allocation_id
        self._longpoll_s = longpoll_s
        self._should_preempt = False
        self._stop = threading.Event()

    def _get_preemption(self, timeout: int) -> bool:
        r = self._session.get(f"/api/v1/allocations/{self._allocation_id}/signals/preemption",
                              params={"timeout_seconds": timeout}, timeout=timeout + 10)
        return bool(r and r.get("preempt"))

    def run(self) -> None:
        try:
            if self._get_preemption(0):
                self._should_preempt = True
                return
            while not self._stop.is_set():
                if self._get_preemption(self._longpoll_s):
                    self._should_preempt = True
                    return
        except Exception as e:  # the master going away must not kill training
            if not self._stop.is_set():
                logger.warning(f"preemption watcher stopped: {e}")

    def close(self) -> None:
        self._stop.set()

    def should_preempt(self) -> bool:
        return self._should_preempt


class PreemptMode(enum.Enum):
    WorkersAskChief = "WORKERS_ASK_CHIEF"
    ChiefOnly = "CHIEF_ONLY"
    ExplicitSignal = "EXPLICIT_SIGNAL"


class PreemptContext:
    def __init__(self, session: Any, allocation_id: str, dist: Any,
                 preempt_mode: PreemptMode = PreemptMode.WorkersAskChief) -> None:
        self._session = session
        self._allocation_id = allocation_id
        self._dist = dist
        self._mode = PreemptMode(preempt_mode)
        self._watcher: Optional[_PreemptionWatcher] = None
        self._ack_sent = False

    def start(self) -> "PreemptContext":
        if self._dist.rank == 0 or self._mode == PreemptMode.ExplicitSignal:
            self._watcher = _PreemptionWatcher(self._session, self._allocation_id)
            self._watcher.start()
        return self

    def close(self) -> None:
        if self._watcher is not None:
            self._watcher.close()

    def __enter__(self) -> "PreemptContext":
        return self.start()

    def __exit__(self, *_: Any) -> None:
        self.close()

    def should_preempt(self, auto_ack: bool = True) -> bool:
        if self._mode == PreemptMode.WorkersAskChief:
            out = self._dist.broadcast(self._watcher.should_preempt() if self._dist.rank == 0 else None)
        elif self._mode == PreemptMode.ChiefOnly:
            if self._dist.rank != 0:
                raise RuntimeError("should_preempt() in ChiefOnly mode may only be called by the chief")
            out = self._watcher.should_preempt() if self._watcher else False
        else:
            out = self._watcher.should_preempt() if self._watcher else False
        if out and auto_ack and self._dist.rank == 0:
            self.acknowledge_preemption_signal()
        return bool(out)

    def acknowledge_preemption_signal(self) -> None:
        if not self._ack_sent:
            self._ack_sent = True
            self._session.post(f"/api/v1/allocations/{self._allocation_id}/signals/ack_preemption")


class DummyPreemptContext(PreemptContext):
    def __init__(self, dist: Any, preempt_mode: PreemptMode = PreemptMode.WorkersAskChief) -> None:
        self._dist = dist
        self._mode = PreemptMode(preempt_mode)
        self._watcher = None
        self._ack_sent = False
        self.flag = False  # tests can set this to simulate a preemption

    def start(self) -> "PreemptContext":
        return self

    def close(self) -> None:
        pass

    def should_preempt(self, auto_ack: bool = True) -> bool:
        if self._mode == PreemptMode.WorkersAskChief:
            return bool(self._dist.broadcast(self.flag if self._dist.rank == 0 else None))
        return self.flag

    def acknowledge_preemption_signal(self) -> None:
        pass
