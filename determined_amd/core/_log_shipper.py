"""Log shipping (reference: ``harness/determined/core/_log_shipper.py``).

On this platform the agent captures each rank's stdout/stderr (prefixed by ``wrap_rank``) and
ships lines to the master itself, so in-process shipping is only used for tasks started
outside an agent with ``DET_SHIP_LOGS=1`` (e.g. unmanaged trials).
"""

import logging
import os
import queue
import sys
import threading
import time
from typing import Any, List, Optional


class _LogShipper:
    def __init__(self, session: Any, task_id: str, rank: int) -> None:
        self._session = session
        self._task_id = task_id
        self._rank = rank
        self._q: "queue.Queue[Optional[str]]" = queue.Queue()
        self._thread = threading.Thread(target=self._run, daemon=True, name="log-shipper")
        self._handler: Optional[logging.Handler] = None

    def start(self) -> None:
        shipper = self

        class H(logging.Handler):
            def emit(self, record: logging.LogRecord) -> None:
                shipper._q.put(self.format(record))

        self._handler = H()
        self._handler.setFormatter(logging.Formatter("%(levelname)s: [%(process)s] %(name)s: %(message)s"))
        logging.getLogger().addHandler(self._handler)
        self._thread.start()

    def _run(self) -> None:
        buf: List[str] = []
        last = time.time()
        while True:
            try:
                item = self._q.get(timeout=1.0)
            except queue.Empty:
                item = ""
            if item is None:
                break
            if item:
                buf.append(item)
            if buf and (len(buf) >= 100 or time.time() - last > 1.0):
                self._flush(buf)
                buf, last = [], time.time()
        if buf:
            self._flush(buf)

    def _flush(self, lines: List[str]) -> None:
        try:
            self._session.post("/api/v1/task/logs", {"task_id": self._task_id,
                                                     "logs": [{"rank": self._rank, "log": ln} for ln in lines]})
        except Exception as e:
            print(f"log shipping failed: {e}", file=sys.stderr)

    def close(self) -> None:
        if self._handler is not None:
            logging.getLogger().removeHandler(self._handler)
        self._q.put(None)
        self._thread.join(timeout=5)


def maybe_log_shipper(session: Any, info: Any, dist: Any) -> Optional[_LogShipper]:
    if os.environ.get("DET_SHIP_LOGS", "0") != "1":
        return None
    return _LogShipper(session, info.task_id, dist.rank)
