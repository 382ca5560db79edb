"""Search methods for DeepSpeed autotuning over the native ZeRO engine (reference:
``harness/determined/pytorch/dsat/_dsat_search_method.py``).

Every trial is a short *profiling run* of the user's DeepSpeedTrial with one candidate
(``zero_optimization.stage``, ``train_micro_batch_size_per_gpu``) written into
``hparams["overwrite_deepspeed_args"]`` and ``hparams["_dsat_mode"] = {...}``: the trial
controller times batches ``start_profile_step..end_profile_step`` and reports the throughput
(samples/s per slot) or latency as its searcher metric, then exits.  A candidate that runs out
of HBM exits early with ``InvalidHP`` (``ExitedReason.INVALID_HP``) -- the search treats that as
"too large" for its stage.

* ``binary``: per ZeRO stage, binary search of the largest micro-batch that fits, each probe
  also giving a throughput sample; stages are searched concurrently.
* ``random``: random (stage, micro-batch) candidates; an OOM at ``m`` removes every ``>= m`` of
  that stage from the pool.
* ``_test``: one micro-batch-1 trial per stage (plumbing check).

The best candidate (and its measured metric) is available as ``best()``; with
``run_full_experiment`` the runner then submits the original experiment with it applied.
"""

import copy
import json
import logging
import pathlib
import random
import uuid
from typing import Any, Dict, List, Optional, Tuple

from determined_amd.pytorch.dsat import defaults
from determined_amd.searcher import (Close, Create, ExitedReason, Operation, Progress, SearcherState,
                                     SearchMethod, Shutdown, ValidateAfter)

logger = logging.getLogger("determined_amd.pytorch.dsat")


class Candidate:
    def __init__(self, stage: int, mbs: int) -> None:
        self.stage = stage
        self.mbs = mbs
        self.metric: Optional[float] = None
        self.oom = False
        self.closed = False

    def to_dict(self) -> Dict[str, Any]:
        return {"stage": self.stage, "mbs": self.mbs, "metric": self.metric, "oom": self.oom, "closed": self.closed}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "Candidate":
        c = cls(int(d["stage"]), int(d["mbs"]))
        c.metric, c.oom, c.closed = d["metric"], d["oom"], d["closed"]
        return c


def candidate_hparams(base_hparams: Dict[str, Any], c: Candidate, start: int, end: int, metric: str) -> Dict[str, Any]:
    hp = copy.deepcopy(base_hparams)
    ow = dict(hp.get(defaults.OVERWRITE_KEY) or {})
    ow["train_micro_batch_size_per_gpu"] = c.mbs
    ow.pop("train_batch_size", None)
    zo = dict(ow.get("zero_optimization") or {})
    zo["stage"] = c.stage
    ow["zero_optimization"] = zo
    hp[defaults.OVERWRITE_KEY] = ow
    hp[defaults.USE_DSAT_MODE_KEY] = {"start_profile_step": start, "end_profile_step": end, "metric": metric}
    return hp


class BaseDSATSearchMethod(SearchMethod):
    def __init__(self, hparams: Dict[str, Any], zero_stages: List[int], max_trials: int, max_concurrent: int,
                 start_profile_step: int = 3, end_profile_step: int = 5, metric: str = "throughput",
                 min_mbs: int = 1, max_mbs: int = 128, seed: int = 42) -> None:
        if metric not in defaults.SMALLER_IS_BETTER_METRICS + defaults.LARGER_IS_BETTER_METRICS:
            raise ValueError(f"unknown dsat metric {metric!r}")
        if end_profile_step <= start_profile_step:
            raise ValueError("end_profile_step must exceed start_profile_step")
        self.hparams = hparams
        self.zero_stages = list(zero_stages)
        self.max_trials = max_trials
        self.max_concurrent = max_concurrent
        self.start, self.end = start_profile_step, end_profile_step
        self.metric_name = metric
        self.smaller_is_better = metric in defaults.SMALLER_IS_BETTER_METRICS
        self.min_mbs, self.max_mbs = min_mbs, max_mbs
        self.rng = random.Random(seed)
        self.trials: Dict[str, Candidate] = {}  # request id -> candidate
        self.queue: List[Candidate] = []
        self.shutdown = False

    # -- bookkeeping -----------------------------------------------------------------------------
    def _running(self) -> int:
        return sum(1 for c in self.trials.values() if not c.closed)

    def _tried(self, stage: int, mbs: int) -> bool:
        return any(c.stage == stage and c.mbs == mbs for c in self.trials.values()) or \
            any(c.stage == stage and c.mbs == mbs for c in self.queue)

    def best(self) -> Optional[Candidate]:
        done = [c for c in self.trials.values() if c.metric is not None]
        if not done:
            return None
        key = (lambda c: c.metric) if self.smaller_is_better else (lambda c: -c.metric)
        return sorted(done, key=lambda c: (key(c), -c.mbs))[0]

    def _launch(self) -> List[Operation]:
        ops: List[Operation] = []
        while self.queue and self._running() < self.max_concurrent and len(self.trials) < self.max_trials:
            c = self.queue.pop(0)
            rid = uuid.uuid4()
            self.trials[str(rid)] = c
            ops.append(Create(rid, candidate_hparams(self.hparams, c, self.start, self.end, self.metric_name)))
            ops.append(ValidateAfter(rid, self.end))
        if not self.shutdown and self._running() == 0 and not self.queue:
            self.shutdown = True
            ops.append(Shutdown())
        elif not self.shutdown and self._running() == 0 and len(self.trials) >= self.max_trials:
            self.shutdown = True
            ops.append(Shutdown())
        return ops

    # -- subclass hooks --------------------------------------------------------------------------
    def initial_candidates(self) -> List[Candidate]:
        raise NotImplementedError

    def next_candidates(self, done: Candidate) -> List[Candidate]:
        raise NotImplementedError

    # -- SearchMethod ----------------------------------------------------------------------------
    def initial_operations(self, searcher_state: SearcherState) -> List[Operation]:
        self.queue = self.initial_candidates()
        return self._launch()

    def on_trial_created(self, searcher_state: SearcherState, request_id: uuid.UUID) -> List[Operation]:
        return []

    def on_validation_completed(self, searcher_state: SearcherState, request_id: uuid.UUID, metric: Any,
                                train_length: int) -> List[Operation]:
        c = self.trials.get(str(request_id))
        if c is None:
            return []
        c.metric = float(metric[self.metric_name] if isinstance(metric, dict) else metric)
        logger.info(f"dsat: stage {c.stage} mbs {c.mbs}: {self.metric_name}={c.metric:.4g}")
        return [Close(request_id)]

    def on_trial_closed(self, searcher_state: SearcherState, request_id: uuid.UUID) -> List[Operation]:
        c = self.trials.get(str(request_id))
        if c is None or c.closed:
            return self._launch()
        c.closed = True
        for n in self.next_candidates(c):
            if not self._tried(n.stage, n.mbs):
                self.queue.append(n)
        return self._launch()

    def on_trial_exited_early(self, searcher_state: SearcherState, request_id: uuid.UUID,
                              exited_reason: ExitedReason) -> List[Operation]:
        c = self.trials.get(str(request_id))
        if c is None:
            return self._launch()
        c.oom = True  # OOM and other failures both mean "does not fit / not viable"
        c.closed = True
        logger.info(f"dsat: stage {c.stage} mbs {c.mbs} exited early ({exited_reason.value})")
        for n in self.next_candidates(c):
            if not self._tried(n.stage, n.mbs):
                self.queue.append(n)
        return self._launch()

    def progress(self, searcher_state: SearcherState) -> float:
        return min(1.0, sum(1 for c in self.trials.values() if c.closed) / max(1, self.max_trials))

    def save_method_state(self, path: pathlib.Path) -> None:
        (path / "dsat_state.json").write_text(json.dumps({
            "trials": {k: v.to_dict() for k, v in self.trials.items()}, "queue": [c.to_dict() for c in self.queue],
            "shutdown": self.shutdown, "extra": self._extra_state()}))

    def load_method_state(self, path: pathlib.Path) -> None:
        d = json.loads((path / "dsat_state.json").read_text())
        self.trials = {k: Candidate.from_dict(v) for k, v in d["trials"].items()}
        self.queue = [Candidate.from_dict(v) for v in d["queue"]]
        self.shutdown = d["shutdown"]
        self._load_extra(d.get("extra") or {})

    def _extra_state(self) -> Dict[str, Any]:
        return {}

    def _load_extra(self, d: Dict[str, Any]) -> None:
        pass

    def summary(self) -> Dict[str, Any]:
        b = self.best()
        return {"best": b.to_dict() if b else None, "metric": self.metric_name,
                "trials": sorted((c.to_dict() for c in self.trials.values()), key=lambda x: (x["stage"], x["mbs"]))}


class BinarySearchDSATSearchMethod(BaseDSATSearchMethod):
    """Per stage: binary search for the largest micro-batch that fits (one probe at a time)."""

    def __init__(self, *a: Any, **kw: Any) -> None:
        super().__init__(*a, **kw)
        self.bounds: Dict[int, Tuple[int, int]] = {s: (self.min_mbs, self.max_mbs) for s in self.zero_stages}

    def _probe(self, stage: int) -> List[Candidate]:
        lo, hi = self.bounds[stage]
        if lo > hi:
            return []
        return [Candidate(stage, (lo + hi + 1) // 2)]

    def initial_candidates(self) -> List[Candidate]:
        out: List[Candidate] = []
        for s in self.zero_stages:
            out += self._probe(s)
        return out

    def next_candidates(self, done: Candidate) -> List[Candidate]:
        lo, hi = self.bounds[done.stage]
        if done.oom:
            hi = min(hi, done.mbs - 1)
        else:
            lo = max(lo, done.mbs + 1)
        self.bounds[done.stage] = (lo, hi)
        return self._probe(done.stage)

    def _extra_state(self) -> Dict[str, Any]:
        return {"bounds": {str(k): list(v) for k, v in self.bounds.items()}}

    def _load_extra(self, d: Dict[str, Any]) -> None:
        if "bounds" in d:
            self.bounds = {int(k): (int(v[0]), int(v[1])) for k, v in d["bounds"].items()}


class RandomDSATSearchMethod(BaseDSATSearchMethod):
    """Random (stage, power-of-two-ish micro-batch) candidates; OOMs prune larger sizes."""

    def __init__(self, *a: Any, **kw: Any) -> None:
        super().__init__(*a, **kw)
        self.cap: Dict[int, int] = {s: self.max_mbs for s in self.zero_stages}

    def _sample(self) -> Optional[Candidate]:
        pool = [(s, m) for s in self.zero_stages for m in range(self.min_mbs, self.cap[s] + 1)
                if not self._tried(s, m)]
        if not pool:
            return None
        s, m = self.rng.choice(pool)
        return Candidate(s, m)

    def initial_candidates(self) -> List[Candidate]:
        out = []
        for _ in range(self.max_concurrent):
            c = self._sample()
            if c is None:
                break
            out.append(c)
            self.queue.append(c)  # so _tried sees it while sampling the rest
        self.queue = []
        return out

    def next_candidates(self, done: Candidate) -> List[Candidate]:
        if done.oom:
            self.cap[done.stage] = min(self.cap[done.stage], done.mbs - 1)
        c = self._sample()
        return [c] if c is not None else []

    def _extra_state(self) -> Dict[str, Any]:
        return {"cap": {str(k): v for k, v in self.cap.items()}}

    def _load_extra(self, d: Dict[str, Any]) -> None:
        if "cap" in d:
            self.cap = {int(k): int(v) for k, v in d["cap"].items()}


class TestDSATSearchMethod(BaseDSATSearchMethod):
    def initial_candidates(self) -> List[Candidate]:
        return [Candidate(s, self.min_mbs) for s in self.zero_stages]

    def next_candidates(self, done: Candidate) -> List[Candidate]:
        return []


METHODS = {"binary": BinarySearchDSATSearchMethod, "random": RandomDSATSearchMethod, "_test": TestDSATSearchMethod}
