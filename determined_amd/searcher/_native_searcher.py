"""Experiment-side searcher: wraps the native C++ search methods with the bookkeeping the
reference keeps in ``master/pkg/searcher/searcher.go`` (request-id <-> trial map, progress,
closed set, snapshot/restore) and the hyperparameter encoding (nested paths, categorical/const
value tables)."""

import copy
from typing import Any, Dict, List, Optional, Set, Tuple

from determined_amd import config as expconf

_TYPES = {"const": 0, "int": 1, "double": 2, "log": 3, "categorical": 4}
EXIT_REASONS = {"errored": 0, "user_canceled": 1, "invalid_hp": 2, "init_invalid_hp": 3, "user_requested_stop": 4}


def flatten_hparams(hps: Dict[str, Any], prefix: str = "") -> Tuple[List[Dict[str, Any]], Dict[str, List[Any]]]:
    """Nested hyperparameter config -> (native spec list, value tables for const/categorical)."""
    flat: List[Dict[str, Any]] = []
    tables: Dict[str, List[Any]] = {}
    for name in sorted(hps):
        hp = expconf.normalize_hparam(hps[name])
        path = prefix + name
        if isinstance(hp, dict) and "type" not in hp:
            f, t = flatten_hparams(hp, path + ".")
            flat += f
            tables.update(t)
            continue
        t = hp["type"]
        spec: Dict[str, Any] = {"path": path, "type": _TYPES[t]}
        if t == "const":
            tables[path] = [hp["val"]]
        elif t == "categorical":
            tables[path] = list(hp["vals"])
            spec["n_vals"] = len(hp["vals"])
        else:
            spec.update(minval=float(hp["minval"]), maxval=float(hp["maxval"]))
            if t == "log":
                spec["base"] = float(hp.get("base", 10))
            if hp.get("count") is not None:
                spec["count"] = int(hp["count"])
        flat.append(spec)
    return flat, tables


def decode_sample(sample: List[Tuple[str, int, int, float]], tables: Dict[str, List[Any]]) -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    for path, kind, i, d in sample:
        val: Any = int(i) if kind == 0 else float(d) if kind == 1 else copy.deepcopy(tables[path][i])
        cur = out
        parts = path.split(".")
        for p in parts[:-1]:
            cur = cur.setdefault(p, {})
        cur[parts[-1]] = val
    return out


class Searcher:
    """One experiment's search state machine (native engine + bookkeeping)."""

    def __init__(self, searcher_cfg: Dict[str, Any], hparams_cfg: Dict[str, Any], seed: int) -> None:
        from determined_amd._native import load

        self.cfg = dict(searcher_cfg)
        self.flat, self.tables = flatten_hparams(hparams_cfg or {})
        eng_cfg = dict(self.cfg)
        if self.cfg.get("max_length") is not None:
            eng_cfg["max_length"] = expconf.Length.parse(self.cfg["max_length"]).units
        for k in ("max_trials", "max_concurrent_trials", "num_rungs", "max_rungs", "divisor"):
            if eng_cfg.get(k) is None:
                eng_cfg.pop(k, None)
        self.engine = load().SearchEngine(eng_cfg, self.flat, int(seed) & ((1 << 63) - 1))
        self.trial_progress: Dict[int, float] = {}
        self.closed: Set[int] = set()
        self.created: Set[int] = set()

    def _decode(self, ops: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
        out = []
        for op in ops:
            op = dict(op)
            if op["type"] == "create":
                op["hparams"] = decode_sample(op["hparams"], self.tables)
            out.append(op)
        return out

    def initial_operations(self) -> List[Dict[str, Any]]:
        return self._decode(self.engine.initial_operations())

    def trial_created(self, request_id: int) -> List[Dict[str, Any]]:
        self.created.add(request_id)
        return self._decode(self.engine.trial_created(request_id))

    def validation_completed(self, request_id: int, metric: float, length: int) -> List[Dict[str, Any]]:
        return self._decode(self.engine.validation_completed(request_id, float(metric), int(length)))

    def trial_closed(self, request_id: int) -> List[Dict[str, Any]]:
        self.closed.add(request_id)
        return self._decode(self.engine.trial_closed(request_id))

    def trial_exited_early(self, request_id: int, reason: str) -> List[Dict[str, Any]]:
        self.closed.add(request_id)
        return self._decode(self.engine.trial_exited_early(request_id, EXIT_REASONS[reason.lower()]))

    def set_trial_progress(self, request_id: int, units: float) -> None:
        self.trial_progress[request_id] = float(units)

    def progress(self) -> float:
        return float(self.engine.progress(self.trial_progress, self.closed))

    def snapshot(self) -> Dict[str, Any]:
        return {"engine": self.engine.snapshot(), "trial_progress": {str(k): v for k, v in self.trial_progress.items()},
                "closed": sorted(self.closed), "created": sorted(self.created)}

    def restore(self, snap: Dict[str, Any]) -> None:
        self.engine.restore(snap["engine"])
        self.trial_progress = {int(k): v for k, v in snap.get("trial_progress", {}).items()}
        self.closed = set(snap.get("closed", []))
        self.created = set(snap.get("created", []))


def simulate(searcher_cfg: Dict[str, Any], hparams_cfg: Dict[str, Any], metric_fn, seed: int = 0,
             max_steps: int = 100000) -> Dict[str, Any]:
    """Run a search to completion against ``metric_fn(hparams, length) -> float`` (reference
    ``master/pkg/searcher/simulate.go``).  Trials run in FIFO order."""
    s = Searcher(searcher_cfg, hparams_cfg, seed)
    queue = list(s.initial_operations())
    trials: Dict[int, Dict[str, Any]] = {}
    pending_validate: Dict[int, List[int]] = {}
    ready: List[int] = []
    steps = 0
    while steps < max_steps:
        steps += 1
        while queue:
            op = queue.pop(0)
            rid = op["request_id"]
            if op["type"] == "create":
                trials[rid] = {"hparams": op["hparams"], "lengths": [], "closed": False, "trained": 0}
                queue += s.trial_created(rid)
            elif op["type"] == "validate_after":
                pending_validate.setdefault(rid, []).append(op["length"])
                if rid not in ready:
                    ready.append(rid)
            elif op["type"] == "close":
                trials[rid]["close_requested"] = True
                if not pending_validate.get(rid):
                    trials[rid]["closed"] = True
                    queue += s.trial_closed(rid)
        if not ready:
            break
        rid = ready.pop(0)
        length = pending_validate[rid].pop(0)
        t = trials[rid]
        t["trained"] = max(t["trained"], length)
        t["lengths"].append(length)
        s.set_trial_progress(rid, length)
        queue += s.validation_completed(rid, metric_fn(t["hparams"], length), length)
        if pending_validate[rid]:
            ready.append(rid)
        elif t.get("close_requested") and not t["closed"]:
            t["closed"] = True
            queue += s.trial_closed(rid)
    return {"trials": trials, "progress": s.progress(), "searcher": s}
