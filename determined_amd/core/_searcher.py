"""SearcherContext (reference: ``harness/determined/core/_searcher.py``).

The chief asks the master for the trial's next operation (train to an absolute ``length``,
then validate and report the searcher metric); with ``WorkersAskChief`` the length is
broadcast so every rank iterates the same operations.
"""

import enum
import logging
from typing import Any, Iterator, Optional

logger = logging.getLogger("determined_amd.core")


class Unit(enum.Enum):
    EPOCHS = "EPOCHS"
    RECORDS = "RECORDS"
    BATCHES = "BATCHES"


def _parse_searcher_units(experiment_config: dict) -> Optional[Unit]:
    s = experiment_config.get("searcher", {}) or {}
    conv = {"records": Unit.RECORDS, "epochs": Unit.EPOCHS, "batches": Unit.BATCHES}
    if s.get("unit"):
        return conv.get(s["unit"])
    ml = s.get("max_length")
    if isinstance(ml, dict) and len(ml) == 1:
        return conv.get(next(iter(ml)))
    return None


class SearcherOperation:
    def __init__(self, session: Any, trial_id: int, length: int, is_chief: bool) -> None:
        self._session = session
        self._trial_id = trial_id
        self._length = length
        self._is_chief = is_chief
        self._completed = False

    @property
    def length(self) -> int:
        return self._length

    def report_progress(self, length: float) -> None:
        if not self._is_chief:
            raise RuntimeError("you must only call op.report_progress() from the chief worker")
        if self._completed and length != self._length:
            raise RuntimeError("you must not call op.report_progress() after op.report_completed()")
        self._session.post(f"/api/v1/trials/{self._trial_id}/progress", {"progress": float(length)})

    def report_completed(self, searcher_metric: Any) -> None:
        if not self._is_chief:
            raise RuntimeError("you must only call op.report_completed() from the chief worker")
        if self._completed:
            raise RuntimeError("you may only call op.report_completed() once")
        self._completed = True
        if hasattr(searcher_metric, "item"):
            searcher_metric = searcher_metric.item()
        self._session.post(f"/api/v1/trials/{self._trial_id}/searcher/completed_operation",
                           {"op": {"length": self._length}, "searcher_metric": searcher_metric})


class SearcherMode(enum.Enum):
    WorkersAskChief = "WORKERS_ASK_CHIEF"
    ChiefOnly = "CHIEF_ONLY"


class SearcherContext:
    def __init__(self, session: Any, dist: Any, trial_id: int, run_id: int, allocation_id: str,
                 units: Optional[Unit] = None) -> None:
        self._session = session
        self._dist = dist
        self._trial_id = trial_id
        self._run_id = run_id
        self._allocation_id = allocation_id
        self._units = units

    def _get_searcher_op(self) -> Optional[SearcherOperation]:
        body = self._session.get(f"/api/v1/trials/{self._trial_id}/searcher/operation")
        if body.get("completed"):
            return None
        length = int(body["op"]["validate_after"]["length"])
        return SearcherOperation(self._session, self._trial_id, length=length, is_chief=self._dist.rank == 0)

    def operations(self, searcher_mode: SearcherMode = SearcherMode.WorkersAskChief,
                   auto_ack: bool = True) -> Iterator[SearcherOperation]:
        searcher_mode = SearcherMode(searcher_mode)
        if self._dist.rank == 0:
            while True:
                op = self._get_searcher_op()
                if searcher_mode == SearcherMode.WorkersAskChief:
                    self._dist.broadcast(op and op.length)
                if op is None:
                    if auto_ack:
                        self.acknowledge_out_of_ops()
                    break
                yield op
                if not op._completed:
                    raise RuntimeError("you must call op.report_completed() on each operation")
        else:
            if searcher_mode != SearcherMode.WorkersAskChief:
                raise RuntimeError("searcher.operations(ChiefOnly) may only be called by the chief")
            while True:
                length = self._dist.broadcast(None)
                if length is None:
                    break
                yield SearcherOperation(self._session, self._trial_id, length=length, is_chief=False)

    def acknowledge_out_of_ops(self) -> None:
        self._session.post(f"/api/v1/allocations/{self._allocation_id}/signals/ack_preemption")

    def get_configured_units(self) -> Optional[Unit]:
        return self._units


class DummySearcherOperation(SearcherOperation):
    def __init__(self, length: int, is_chief: bool) -> None:
        self._length = length
        self._is_chief = is_chief
        self._completed = False
        self.metric: Any = None

    def report_progress(self, length: float) -> None:
        if not self._is_chief:
            raise RuntimeError("you must only call op.report_progress() from the chief worker")
        logger.info(f"progress report: {length}/{self._length}")

    def report_completed(self, searcher_metric: Any) -> None:
        if not self._is_chief:
            raise RuntimeError("you must only call op.report_completed() from the chief worker")
        if self._completed:
            raise RuntimeError("you may only call op.report_completed() once")
        self._completed = True
        self.metric = searcher_metric
        logger.info(f"SearcherOperation complete: searcher_metric={searcher_metric}")


class DummySearcherContext(SearcherContext):
    """Yields one operation of ``length`` (default 1) off-cluster."""

    def __init__(self, dist: Any, length: int = 1) -> None:
        self._dist = dist
        self._length = length

    def operations(self, searcher_mode: SearcherMode = SearcherMode.WorkersAskChief,
                   auto_ack: bool = True) -> Iterator[SearcherOperation]:
        searcher_mode = SearcherMode(searcher_mode)
        if self._dist.rank == 0:
            op = DummySearcherOperation(self._length, True)
            if searcher_mode == SearcherMode.WorkersAskChief:
                self._dist.broadcast(op.length)
            yield op
            if not op._completed:
                raise RuntimeError("you must call op.report_completed() on each operation")
            if searcher_mode == SearcherMode.WorkersAskChief:
                self._dist.broadcast(None)
        else:
            if searcher_mode != SearcherMode.WorkersAskChief:
                raise RuntimeError("searcher.operations(ChiefOnly) may only be called by the chief")
            while True:
                length = self._dist.broadcast(None)
                if length is None:
                    break
                yield DummySearcherOperation(length, False)

    def acknowledge_out_of_ops(self) -> None:
        pass

    def get_configured_units(self) -> Optional[Unit]:
        return Unit.EPOCHS
