"""Metric reducers (reference: ``harness/determined/pytorch/_reducer.py``)."""

import abc
import enum
from typing import Any, Callable, Dict, List, Optional, Union

import numpy as np


class Reducer(enum.Enum):
    AVG = 1
    SUM = 2
    MAX = 3
    MIN = 4


def _simple_reduce_metrics(reducer: Reducer, metrics: List[Any], num_batches: Optional[List[int]] = None) -> Any:
    arr = np.asarray([np.asarray(m, dtype=np.float64) for m in metrics])
    if reducer == Reducer.AVG:
        if num_batches is not None and len(num_batches) == len(metrics):
            w = np.asarray(num_batches, dtype=np.float64)
            return float(np.average(arr, weights=w, axis=0)) if arr.ndim == 1 else np.average(arr, weights=w, axis=0)
        return np.mean(arr, axis=0)
    if reducer == Reducer.SUM:
        return np.sum(arr, axis=0)
    if reducer == Reducer.MAX:
        return np.max(arr, axis=0)
    if reducer == Reducer.MIN:
        return np.min(arr, axis=0)
    raise NotImplementedError(reducer)


class MetricReducer(metaclass=abc.ABCMeta):
    """Custom reducer: ``update()`` per batch, ``per_slot_reduce()`` per rank,
    ``cross_slot_reduce(list)`` on the chief."""

    @abc.abstractmethod
    def reset(self) -> None:
        pass

    @abc.abstractmethod
    def per_slot_reduce(self) -> Any:
        pass

    @abc.abstractmethod
    def cross_slot_reduce(self, per_slot_metrics: List[Any]) -> Any:
        pass


class _SimpleReducer(MetricReducer):
    def __init__(self, fn: Callable[[List[Any]], Any]) -> None:
        self.fn = fn
        self.reset()

    def reset(self) -> None:
        self.updates: List[Any] = []

    def update(self, value: Any) -> None:
        self.updates.append(value)

    def per_slot_reduce(self) -> Any:
        return self.updates

    def cross_slot_reduce(self, per_slot_metrics: List[Any]) -> Any:
        flat = [v for slot in per_slot_metrics for v in slot]
        return self.fn(flat)


class _WrappedReducer:
    def __init__(self, reducer: MetricReducer, name: Optional[str]) -> None:
        self.reducer = reducer
        self.name = name


class _PyTorchReducerContext:
    def __init__(self, allgather_fn: Optional[Callable[[Any], List[Any]]] = None) -> None:
        self._wrapped_reducers: List[_WrappedReducer] = []
        self._allgather_fn = allgather_fn or (lambda x: [x])

    def reset_reducers(self) -> None:
        for w in self._wrapped_reducers:
            w.reducer.reset()

    def wrap_reducer(self, reducer: Union[Callable, MetricReducer], name: Optional[str] = None,
                     for_training: bool = True, for_validation: bool = True) -> MetricReducer:
        if not isinstance(reducer, MetricReducer):
            reducer = _SimpleReducer(reducer)
        w = _WrappedReducer(reducer, name)
        w.for_training, w.for_validation = for_training, for_validation  # type: ignore[attr-defined]
        self._wrapped_reducers.append(w)
        return reducer

    def reduce_metrics(self, for_training: bool) -> Dict[str, Any]:
        out: Dict[str, Any] = {}
        for w in self._wrapped_reducers:
            if not getattr(w, "for_training" if for_training else "for_validation", True):
                continue
            per_slot = self._allgather_fn(w.reducer.per_slot_reduce())
            val = w.reducer.cross_slot_reduce(per_slot)
            if w.name is None:
                if not isinstance(val, dict):
                    raise ValueError("an unnamed reducer must return a dict of metrics")
                out.update(val)
            else:
                out[w.name] = val
        return out
