"""The master's state machines (reference: ``master/internal/{experiment,trial,checkpoint_gc}.go``,
``master/internal/task`` allocations/preemption, ``master/internal/rm/agentrm`` resource manager).

One process, one global lock.  Experiments own a searcher (native C++ engine or a custom
searcher event queue); each searcher ``create`` becomes a trial, each ``validate_after`` is
queued on its trial, ``close`` ends it.  Trials with work and no allocation request slots from
the native scheduler; allocations are dispatched to agents, which launch the harness.
"""

import base64
import json
import re
import logging
import os
import threading
import time
import uuid
from typing import Any, Dict, List, Optional, Tuple

from determined_amd import config as expconf
from determined_amd.master._db import DB

logger = logging.getLogger("determined_amd.master")

TERMINAL_EXP = {"COMPLETED", "CANCELED", "ERROR", "DELETED"}
TERMINAL_TRIAL = {"COMPLETED", "CANCELED", "ERROR"}


class Allocation:
    def __init__(self, alloc_id: str, task_id: str, slots: int, exp_id: Optional[int] = None,
                 trial_id: Optional[int] = None, kind: str = "TRIAL") -> None:
        self.id = alloc_id
        self.task_id = task_id
        self.slots = slots
        self.exp_id = exp_id
        self.trial_id = trial_id
        self.kind = kind
        self.state = "PENDING"
        self.assignment: List[Tuple[str, List[int]]] = []
        self.preempt = False
        self.ack_preempt = False
        self.killed = False
        self.exit_codes: Dict[str, int] = {}
        self.start_time = time.time()
        # all-gather rounds: the forming round (request_uuid -> (order key, data)) and the results
        # + member uuids of the last completed rounds (a repeat post is an idempotent re-fetch)
        self.gather: Dict[str, Tuple[Any, Any]] = {}
        self.gather_round = 0
        self.gather_done: Dict[int, Tuple[List[Any], frozenset]] = {}

    def to_dict(self) -> Dict[str, Any]:
        return {"allocation_id": self.id, "task_id": self.task_id, "slots": self.slots, "state": self.state,
                "assignment": self.assignment, "preempt": self.preempt, "killed": self.killed,
                "trial_id": self.trial_id, "experiment_id": self.exp_id}


class TrialRec:
    def __init__(self, tid: int, exp_id: int, request_id: int, hparams: Dict[str, Any], seed: int) -> None:
        self.id = tid
        self.exp_id = exp_id
        self.request_id = request_id
        self.hparams = hparams
        self.seed = seed
        self.state = "ACTIVE"
        self.ops: List[int] = []
        self.close_requested = False
        self.restarts = 0
        self.run_id = 0
        self.allocation: Optional[Allocation] = None
        self.latest_checkpoint: Optional[str] = None
        self.total_batches = 0
        self.early_exit: Optional[str] = None
        self.warm_start: Optional[str] = None
        self.no_retry = False                  # log policy cancel_retries matched
        self.excluded_agents: List[str] = []  # log policy exclude_node matched
        self.last_activity: Optional[float] = None  # unmanaged trials: last state report / heartbeat

    def searcher_state(self) -> Dict[str, Any]:
        return {"ops": self.ops, "close_requested": self.close_requested, "early_exit": self.early_exit}


class ExperimentRec:
    def __init__(self, eid: int, cfg: Dict[str, Any], state: str) -> None:
        self.deferred: List["TrialRec"] = []  # trials waiting for resources.max_slots
        self.id = eid
        self.config = cfg
        self.state = state
        self.searcher: Any = None
        self.custom_events: List[Dict[str, Any]] = []
        self.custom_event_id = 0
        self.trials: Dict[int, TrialRec] = {}  # request_id -> trial
        self.shutdown = False
        self.progress = 0.0


class Master:
    def __init__(self, db_path: str = ":memory:", policy: str = "priority", fit: str = "best",
                 preemption: bool = True, cluster_id: Optional[str] = None, master_url: str = "http://127.0.0.1:8080",
                 auth_token: Optional[str] = None, auth: str = "none",
                 resource_pools: Optional[List[Dict[str, Any]]] = None, default_compute_pool: Optional[str] = None,
                 default_aux_pool: Optional[str] = None) -> None:
        from determined_amd._native import load
        from determined_amd.master._iam import IAM
        from determined_amd.master._pools import PoolSet, parse_pools

        self.native = load()
        self.lock = threading.RLock()
        self.cv = threading.Condition(self.lock)
        self.db = DB(db_path)
        self.iam = IAM(self.db, mode=auth, cluster_token=auth_token)
        self.policy = policy
        self.fit = fit
        # one native scheduler per resource pool (master/_pools.py); a single "default" pool
        # with the master-wide policy unless the config lists pools
        self.sched = PoolSet(self.native, parse_pools(resource_pools, policy, fit, preemption),
                             default_compute_pool, default_aux_pool)
        self.cluster_id = cluster_id or str(uuid.uuid4())
        self.master_url = master_url
        self.auth_token = auth_token
        self.agents: Dict[str, Dict[str, Any]] = {}
        self.allocations: Dict[str, Allocation] = {}
        self.experiments: Dict[int, ExperimentRec] = {}
        self._order = 0
        self._closed = False
        self._init_stream()
        self._restore()
        self._ticker = threading.Thread(target=self._tick_loop, daemon=True, name="master-tick")
        self._ticker.start()

    # ================================================================ lifecycle / restore
    def close(self) -> None:
        with self.lock:
            self._closed = True
            self.cv.notify_all()
        with self.stream_cv:
            self.stream_cv.notify_all()

    # ================================================================ event stream
    # Reference: master/internal/stream (websocket subscriptions to entity changes).  Every write to
    # a streamed table (_db.STREAMED) becomes an event {seq, ts, entity, id, fields}; clients long-poll
    # GET /api/v1/stream?since=<seq> and get the newer events (or resync=true once the ring has
    # dropped what they missed).  Large columns (configs, model definitions, snapshots) stay out.
    _STREAM_SKIP = {"config", "model_def", "searcher_snapshot", "searcher_state", "metadata", "resources",
                    "batch_metrics", "proxy"}

    def _init_stream(self, capacity: int = 20000) -> None:
        import collections

        self.stream_cv = threading.Condition()
        self.stream_events: "collections.deque" = collections.deque(maxlen=capacity)
        self.stream_seq = 0
        # per-process epoch: a client that echoes another process's epoch (the master restarted and
        # its sequence started over) is told to resync whatever its `since`
        self.stream_epoch = uuid.uuid4().hex[:12]

        def on_change(table: str, key: Any, cols: Dict[str, Any]) -> None:
            from determined_amd.master._db import STREAMED

            fields = {k: v for k, v in cols.items() if k not in self._STREAM_SKIP and not isinstance(v, bytes)}
            if table == "metrics":
                key = cols.get("trial_id")
            with self.stream_cv:
                self.stream_seq += 1
                self.stream_events.append({"seq": self.stream_seq, "ts": time.time(), "entity": STREAMED[table],
                                           "id": key, "fields": fields})
                self.stream_cv.notify_all()

        self.db.on_change = on_change

    def stream(self, since: int, timeout: float = 0.0, entities: Optional[List[str]] = None,
               epoch: Optional[str] = None) -> Dict[str, Any]:
        """Events after ``since``; ``resync=True`` when the client cannot catch up incrementally:
        the ring dropped what it missed, its ``since`` is ahead of this process's sequence, or it
        echoes the ``epoch`` of an earlier master process."""
        deadline = time.time() + timeout
        with self.stream_cv:
            while True:
                head = {"last_seq": self.stream_seq, "epoch": self.stream_epoch}
                oldest = self.stream_events[0]["seq"] if self.stream_events else self.stream_seq + 1
                if ((since + 1 < oldest and since < self.stream_seq) or since > self.stream_seq
                        or (epoch and epoch != self.stream_epoch)):
                    return {"events": [], "resync": True, **head}
                evs = [e for e in self.stream_events if e["seq"] > since and (not entities or e["entity"] in entities)]
                if evs or time.time() >= deadline or self._closed:
                    return {"events": evs, "resync": False, **head}
                self.stream_cv.wait(max(0.0, min(1.0, deadline - time.time())))

    def _tick_loop(self) -> None:
        last_cleanup = 0.0
        while True:
            with self.lock:
                if self._closed:
                    return
                self._check_agents()
                self._reap_unmanaged()
                self._schedule()
                if time.time() - last_cleanup > 600:
                    last_cleanup = time.time()
                    try:
                        self.cleanup_logs()
                    except Exception as e:  # retention is best effort
                        logger.warning(f"log retention cleanup failed: {e}")
                self.cv.wait(1.0)

    def _restore(self) -> None:
        for row in self.db.all("SELECT * FROM experiments WHERE state IN ('ACTIVE','PAUSED','STOPPING_CANCELED',"
                               "'STOPPING_COMPLETED')"):
            cfg = row["config"]
            exp = ExperimentRec(row["id"], cfg, row["state"])
            self.experiments[exp.id] = exp
            if row.get("unmanaged"):
                exp.unmanaged = True  # type: ignore[attr-defined]
            elif cfg["searcher"]["name"] != "custom":
                from determined_amd.searcher import Searcher

                exp.searcher = Searcher(cfg["searcher"], cfg.get("hyperparameters", {}),
                                        cfg["reproducibility"]["experiment_seed"])
                if row.get("searcher_snapshot"):
                    exp.searcher.restore(row["searcher_snapshot"])
            for t in self.db.all("SELECT * FROM trials WHERE experiment_id=?", [exp.id]):
                tr = TrialRec(t["id"], exp.id, t["request_id"], t["hparams"], t["seed"])
                tr.state = t["state"]
                tr.restarts = t["restarts"] or 0
                tr.run_id = t["run_id"] or 0
                tr.latest_checkpoint = t["latest_checkpoint"]
                tr.total_batches = t["total_batches"] or 0
                ss = t.get("searcher_state") or {}
                tr.ops = list(ss.get("ops", []))
                tr.close_requested = bool(ss.get("close_requested", False))
                tr.early_exit = ss.get("early_exit")
                tr.warm_start = t.get("warm_start_checkpoint")
                exp.trials[tr.request_id] = tr
                if exp.state == "ACTIVE" and tr.state == "ACTIVE" and tr.ops:
                    self._request_allocation(exp, tr)
            self._order = max(self._order, exp.id * 1000)

    # ================================================================ experiments
    def create_experiment(self, cfg: Dict[str, Any], model_def: Optional[bytes], activate: bool = True,
                          parent_id: Optional[int] = None, unmanaged: bool = False) -> int:
        cfg = expconf.parse(cfg)
        with self.lock:
            res = cfg["resources"]
            res["resource_pool"] = self.check_pool(res.get("resource_pool"), int(res.get("slots_per_trial", 1)),
                                                   cfg.get("workspace") or "Uncategorized")
            eid = self.db.insert("experiments", name=cfg["name"], state="ACTIVE" if activate else "PAUSED",
                                 config=cfg, model_def=model_def, parent_id=parent_id, start_time=time.time(),
                                 description=cfg.get("description") or "", labels=cfg.get("labels") or [],
                                 unmanaged=int(unmanaged), project=cfg.get("project") or "Uncategorized",
                                 workspace=cfg.get("workspace") or "Uncategorized",
                                 owner=self.iam.current()["username"])
            exp = ExperimentRec(eid, cfg, "ACTIVE" if activate else "PAUSED")
            self.experiments[eid] = exp
            if cfg["searcher"]["name"] == "custom":
                self._custom_event(exp, {"initial_operations": {}})
            else:
                from determined_amd.searcher import Searcher

                exp.searcher = Searcher(cfg["searcher"], cfg.get("hyperparameters", {}),
                                        cfg["reproducibility"]["experiment_seed"])
                self._process_ops(exp, exp.searcher.initial_operations())
            self._persist_exp(exp)
            self._fire_webhooks(exp, "EXPERIMENT_STATE_CHANGE")
            self.cv.notify_all()
            return eid

    # ---------------------------------------------------------------- unmanaged (core_v2)
    def create_unmanaged_experiment(self, cfg: Dict[str, Any], external_id: Optional[str] = None) -> int:
        """Experiment whose trials run outside the cluster and only report (no searcher, no
        allocations); ``external_id`` makes the call idempotent (resume / multi-trial grouping)."""
        with self.lock:
            if external_id:
                row = self.db.one("SELECT id FROM experiments WHERE external_id=?", [external_id])
                if row is not None:
                    return int(row["id"])
            cfg = dict(cfg)
            cfg.setdefault("entrypoint", "unmanaged")
            cfg = expconf.parse(cfg)
            eid = self.db.insert("experiments", name=cfg["name"], state="ACTIVE", config=cfg, model_def=None,
                                 start_time=time.time(), description=cfg.get("description") or "",
                                 labels=cfg.get("labels") or [], unmanaged=1, external_id=external_id,
                                 project=cfg.get("project") or "Uncategorized",
                                 workspace=cfg.get("workspace") or "Uncategorized")
            exp = ExperimentRec(eid, cfg, "ACTIVE")
            exp.unmanaged = True  # type: ignore[attr-defined]
            self.experiments[eid] = exp
            return eid

    def create_unmanaged_trial(self, eid: int, hparams: Dict[str, Any],
                               external_id: Optional[str] = None) -> Dict[str, Any]:
        with self.lock:
            exp = self.experiments.get(eid)
            if exp is None:  # finished earlier (or before a master restart): re-register to resume
                exp = self._exp(eid)
                exp.unmanaged = True  # type: ignore[attr-defined]
                for t in self.db.all("SELECT * FROM trials WHERE experiment_id=?", [eid]):
                    tr = TrialRec(t["id"], eid, t["request_id"], t["hparams"], t["seed"])
                    tr.state, tr.total_batches = t["state"], t["total_batches"] or 0
                    tr.latest_checkpoint = t["latest_checkpoint"]
                    exp.trials[tr.request_id] = tr
                self.experiments[eid] = exp
            if external_id:
                row = self.db.one("SELECT * FROM trials WHERE experiment_id=? AND external_id=?", [eid, external_id])
                if row is not None:
                    tr = next((t for t in exp.trials.values() if t.id == row["id"]), None)
                    if tr is not None and tr.state in TERMINAL_TRIAL:
                        tr.state = "ACTIVE"  # resumed
                        self._persist_trial(tr)
                    if exp.state in TERMINAL_EXP:
                        exp.state = "ACTIVE"
                        self.db.update("experiments", "id", eid, state="ACTIVE", end_time=None)
                    return {"trial_id": row["id"], "latest_checkpoint": row.get("latest_checkpoint"),
                            "steps_completed": row.get("total_batches") or 0}
            rid = len(exp.trials) + 1
            while rid in exp.trials:
                rid += 1
            seed = (exp.config["reproducibility"]["experiment_seed"] + rid) % (2**31)
            tid = self.db.insert("trials", experiment_id=eid, request_id=rid, state="ACTIVE", hparams=hparams or {},
                                 seed=seed, start_time=time.time(), external_id=external_id)
            tr = TrialRec(tid, eid, rid, hparams or {}, seed)
            exp.trials[rid] = tr
            return {"trial_id": tid, "latest_checkpoint": None, "steps_completed": 0}

    # an unmanaged trial whose chief stopped sending heartbeats for this long is marked ERROR
    unmanaged_timeout_s = float(os.environ.get("DET_UNMANAGED_TIMEOUT_S", "600"))

    def unmanaged_trial_report(self, tid: int, state: Optional[str]) -> None:
        """``PATCH /api/v1/trials/<id>`` from an unmanaged trial's heartbeat: RUNNING on start,
        bare heartbeats while it runs, COMPLETED / ERROR / CANCELED at the end."""
        with self.lock:
            exp, tr = self._trial(tid)
            if not getattr(exp, "unmanaged", False):
                raise ValueError(f"trial {tid} is managed by the master: its state is not reported by the trial")
            tr.last_activity = time.time()
            if state is None:
                return
            state = str(state).upper()
            if state == "RUNNING":
                if tr.state in TERMINAL_TRIAL:  # a resumed run
                    tr.state = "ACTIVE"
                    self._persist_trial(tr)
                if exp.state in TERMINAL_EXP:
                    exp.state = "ACTIVE"
                    self.db.update("experiments", "id", exp.id, state="ACTIVE", end_time=None)
                return
            if state not in TERMINAL_TRIAL:
                raise ValueError(f"unknown trial state {state!r}")
            tr.last_activity = None
        self.close_unmanaged_trial(tid, state)

    def _reap_unmanaged(self) -> None:
        """Unmanaged trials that reported a heartbeat once and then went silent for longer than
        ``unmanaged_timeout_s`` (the process was killed, its host died) end in ERROR."""
        now = time.time()
        for exp in list(self.experiments.values()):
            if not getattr(exp, "unmanaged", False):
                continue
            for tr in list(exp.trials.values()):
                if tr.state not in TERMINAL_TRIAL and tr.last_activity is not None and \
                        now - tr.last_activity > self.unmanaged_timeout_s:
                    logger.warning(f"unmanaged trial {tr.id}: no heartbeat for {now - tr.last_activity:.0f} s, ERROR")
                    tr.last_activity = None
                    tr.state = "ERROR"
                    self._persist_trial(tr)
                    if all(t.state in TERMINAL_TRIAL for t in exp.trials.values()):
                        self._set_exp_state(exp, "ERROR" if all(t.state == "ERROR" for t in exp.trials.values())
                                            else "COMPLETED")

    def close_unmanaged_trial(self, tid: int, state: str = "COMPLETED") -> None:
        with self.lock:
            exp, tr = self._trial(tid)
            tr.state = state if state in TERMINAL_TRIAL else "COMPLETED"
            self._persist_trial(tr)
            if all(t.state in TERMINAL_TRIAL for t in exp.trials.values()):
                self._set_exp_state(exp, "ERROR" if all(t.state == "ERROR" for t in exp.trials.values())
                                    else "COMPLETED")

    def _persist_exp(self, exp: ExperimentRec) -> None:
        snap = exp.searcher.snapshot() if exp.searcher is not None else None
        if exp.searcher is not None:
            try:
                exp.progress = exp.searcher.progress()
            except Exception:
                pass
        self.db.update("experiments", "id", exp.id, state=exp.state, searcher_snapshot=snap, progress=exp.progress)

    def _persist_trial(self, tr: TrialRec) -> None:
        self.db.update("trials", "id", tr.id, state=tr.state, restarts=tr.restarts, run_id=tr.run_id,
                       latest_checkpoint=tr.latest_checkpoint, total_batches=tr.total_batches,
                       searcher_state=tr.searcher_state(),
                       end_time=time.time() if tr.state in TERMINAL_TRIAL else None)

    def _process_ops(self, exp: ExperimentRec, ops: List[Dict[str, Any]]) -> None:
        """Apply searcher operations (reference experiment.go:processOperations)."""
        queue = list(ops)
        while queue:
            op = queue.pop(0)
            t = op["type"]
            rid = op.get("request_id")
            if t == "create":
                seed = (exp.config["reproducibility"]["experiment_seed"] + len(exp.trials)) % (2**31)
                tid = self.db.insert("trials", experiment_id=exp.id, request_id=rid, state="ACTIVE",
                                     hparams=op["hparams"], seed=seed, start_time=time.time(),
                                     warm_start_checkpoint=op.get("checkpoint"))
                tr = TrialRec(tid, exp.id, rid, op["hparams"], seed)
                tr.warm_start = op.get("checkpoint") or exp.config["searcher"].get("source_checkpoint_uuid")
                exp.trials[rid] = tr
                if exp.searcher is not None:
                    queue += exp.searcher.trial_created(rid)
                else:
                    self._custom_event(exp, {"trial_created": {"request_id": rid}})
            elif t == "validate_after":
                tr = exp.trials.get(rid)
                if tr is None or tr.state in TERMINAL_TRIAL:
                    continue
                tr.ops.append(int(op["length"]))
                self._persist_trial(tr)
                if tr.allocation is None and exp.state == "ACTIVE":
                    self._request_allocation(exp, tr)
            elif t == "close":
                tr = exp.trials.get(rid)
                if tr is None or tr.state in TERMINAL_TRIAL:
                    continue
                tr.close_requested = True
                self._persist_trial(tr)
                if tr.allocation is None and not tr.ops:
                    queue += self._finish_trial(exp, tr, "COMPLETED")
            elif t == "shutdown":
                exp.shutdown = True
                if op.get("cancel"):
                    self._stop_experiment(exp, "CANCELED")
                elif op.get("failure"):
                    self._stop_experiment(exp, "ERROR")
            elif t == "progress":
                exp.progress = float(op.get("progress", 0.0))
        self._maybe_complete(exp)
        self._persist_exp(exp)

    def _finish_trial(self, exp: ExperimentRec, tr: TrialRec, state: str) -> List[Dict[str, Any]]:
        if tr.state in TERMINAL_TRIAL:
            return []
        tr.state = state
        self._persist_trial(tr)
        self._fire_webhooks(exp, "TRIAL_STATE_CHANGE", trial=tr)
        if exp.searcher is None:
            if state == "COMPLETED" and not tr.early_exit:
                self._custom_event(exp, {"trial_closed": {"request_id": tr.request_id}})
            else:
                self._custom_event(exp, {"trial_exited_early": {"request_id": tr.request_id,
                                                                "exited_reason": tr.early_exit or "errored"}})
            return []
        if state == "COMPLETED" and not tr.early_exit:
            return exp.searcher.trial_closed(tr.request_id)
        reason = tr.early_exit or ("user_canceled" if state == "CANCELED" else "errored")
        return exp.searcher.trial_exited_early(tr.request_id, reason)

    def _maybe_complete(self, exp: ExperimentRec) -> None:
        if exp.state in TERMINAL_EXP:
            return
        active = [t for t in exp.trials.values() if t.state not in TERMINAL_TRIAL]
        if exp.state in ("STOPPING_CANCELED", "STOPPING_ERROR") and not any(t.allocation for t in active):
            for t in active:
                t.state = "CANCELED"
                self._persist_trial(t)
            self._set_exp_state(exp, "CANCELED" if exp.state == "STOPPING_CANCELED" else "ERROR")
            return
        if exp.searcher is None and not exp.shutdown:
            return
        if not active and exp.trials:
            all_err = all(t.state == "ERROR" for t in exp.trials.values())
            self._set_exp_state(exp, "ERROR" if all_err else "COMPLETED")
        elif exp.shutdown and not active:
            self._set_exp_state(exp, "COMPLETED")

    def _set_exp_state(self, exp: ExperimentRec, state: str) -> None:
        exp.state = state
        self.db.update("experiments", "id", exp.id, state=state,
                       end_time=time.time() if state in TERMINAL_EXP else None)
        self._fire_webhooks(exp, "EXPERIMENT_STATE_CHANGE")
        if state in TERMINAL_EXP:
            exp.progress = 1.0 if state == "COMPLETED" else exp.progress
            self._persist_exp(exp)
            threading.Thread(target=self.gc_experiment_checkpoints, args=(exp.id,), daemon=True).start()
            self._custom_event(exp, {"experiment_inactive": {"experiment_state": state}})
        self.cv.notify_all()

    def _stop_experiment(self, exp: ExperimentRec, final: str) -> None:
        exp.state = "STOPPING_CANCELED" if final == "CANCELED" else "STOPPING_ERROR"
        for tr in exp.trials.values():
            if tr.allocation is not None:
                self._kill_allocation(tr.allocation)
        self._maybe_complete(exp)

    def pause_experiment(self, eid: int) -> None:
        with self.lock:
            exp = self._exp(eid)
            if exp.state != "ACTIVE":
                return
            self._set_exp_state(exp, "PAUSED")
            for tr in exp.trials.values():
                a = tr.allocation
                if a is not None:
                    if a.state == "PENDING":
                        self._drop_allocation(a)
                        tr.allocation = None
                    else:
                        a.preempt = True
            self.cv.notify_all()

    def activate_experiment(self, eid: int) -> None:
        with self.lock:
            exp = self._exp(eid)
            if exp.state != "PAUSED":
                return
            self._set_exp_state(exp, "ACTIVE")
            for tr in exp.trials.values():
                if tr.state == "ACTIVE" and tr.ops and tr.allocation is None:
                    self._request_allocation(exp, tr)
            self.cv.notify_all()

    def kill_experiment(self, eid: int) -> None:
        with self.lock:
            exp = self._exp(eid)
            if exp.state in TERMINAL_EXP:
                return
            self._stop_experiment(exp, "CANCELED")
            self.cv.notify_all()

    def archive_experiment(self, eid: int, archived: bool = True) -> None:
        with self.lock:
            self.db.update("experiments", "id", eid, archived=int(archived))

    def delete_experiment(self, eid: int) -> None:
        with self.lock:
            exp = self.experiments.get(eid)
            if exp is not None and exp.state not in TERMINAL_EXP:
                raise ValueError("only terminal experiments can be deleted")
            self.gc_experiment_checkpoints(eid, delete_all=True)
            self.db.update("experiments", "id", eid, state="DELETED")

    def _exp(self, eid: int) -> ExperimentRec:
        exp = self.experiments.get(eid)
        if exp is None:
            row = self.db.one("SELECT id, state, config FROM experiments WHERE id=?", [eid])
            if row is None:
                raise KeyError(f"experiment {eid} not found")
            exp = ExperimentRec(eid, row["config"], row["state"])
        return exp

    def _trial(self, tid: int) -> Tuple[ExperimentRec, TrialRec]:
        for exp in self.experiments.values():
            for tr in exp.trials.values():
                if tr.id == tid:
                    return exp, tr
        raise KeyError(f"trial {tid} not active")

    # ================================================================ allocations
    def _next_order(self) -> int:
        self._order += 1
        return self._order

    def _exp_slots_in_use(self, exp: ExperimentRec) -> int:
        return sum(a.slots for a in self.allocations.values() if a.exp_id == exp.id and a.state != "TERMINATED")

    def _request_allocation(self, exp: ExperimentRec, tr: TrialRec) -> None:
        slots = int(exp.config["resources"].get("slots_per_trial", 1))
        cap = exp.config["resources"].get("max_slots")
        if cap is not None and self._exp_slots_in_use(exp) + slots > int(cap):
            # resources.max_slots: queue the trial in the master until the experiment frees slots
            if tr not in exp.deferred:
                exp.deferred.append(tr)
            return
        self._start_request(exp, tr, slots)

    def _drain_deferred(self, exp: ExperimentRec) -> None:
        cap = exp.config["resources"].get("max_slots")
        slots = int(exp.config["resources"].get("slots_per_trial", 1))
        while exp.deferred and exp.state == "ACTIVE":
            if cap is not None and self._exp_slots_in_use(exp) + slots > int(cap):
                return
            tr = exp.deferred.pop(0)
            if tr.state not in TERMINAL_TRIAL and tr.allocation is None:
                self._start_request(exp, tr, slots)

    def _start_request(self, exp: ExperimentRec, tr: TrialRec, slots: int) -> None:
        aid = f"trial-{tr.id}.{tr.run_id + 1}.{uuid.uuid4().hex[:6]}"
        a = Allocation(aid, f"trial-{tr.id}", slots, exp.id, tr.id)
        a.progress_at_start = (tr.total_batches, len(tr.ops))  # type: ignore[attr-defined]
        tr.allocation = a
        self.allocations[aid] = a
        prio = exp.config["resources"].get("priority")
        self.sched.set_max_slots(f"exp-{exp.id}", exp.config["resources"].get("max_slots"))
        self.sched.add_request(aid, f"exp-{exp.id}", slots, int(prio) if prio is not None else 42,
                               float(exp.config["resources"].get("weight", 1)), self._next_order(), True,
                               list(tr.excluded_agents), pool=exp.config["resources"].get("resource_pool") or None)
        self.cv.notify_all()

    def create_command(self, cmd: List[str], slots: int = 0, env: Optional[Dict[str, str]] = None,
                       kind: str = "COMMAND", workdir_b64: Optional[str] = None,
                       resource_pool: Optional[str] = None, priority: Optional[int] = None,
                       workspace_id: Optional[int] = None, task_config: Optional[Dict[str, Any]] = None) -> str:
        """``task_config``: the expconf sections a command's container honours (environment,
        bind_mounts, resources) -- shipped to the agent as DET_TASK_CONFIG."""
        with self.lock:
            pool = self.check_pool(resource_pool, slots, None)
            task_id = f"{kind.lower()}-{uuid.uuid4().hex[:8]}"
            aid = f"{task_id}.1"
            a = Allocation(aid, task_id, slots, kind=kind)
            a.command = cmd  # type: ignore[attr-defined]
            a.env = env or {}  # type: ignore[attr-defined]
            a.workdir_b64 = workdir_b64  # type: ignore[attr-defined]
            a.task_config = task_config or None  # type: ignore[attr-defined]
            self.allocations[aid] = a
            owner = self.iam.current() if self.iam is not None else None
            self.db.insert("tasks", id=task_id, type=kind, state="PENDING",
                           config={"cmd": cmd, "slots": slots, "resource_pool": pool,
                                   "priority": 42 if priority is None else int(priority),
                                   # who may reach the task's service through the master's proxy
                                   "owner_id": owner["id"] if owner else None,
                                   "workspace_id": workspace_id},
                           start_time=time.time())
            self.sched.add_request(aid, task_id, slots, 42 if priority is None else int(priority), 1.0,
                                   self._next_order(), False, pool=pool)
            self.cv.notify_all()
            return task_id

    def set_task_priority(self, task_id: str, priority: Optional[int] = None, weight: Optional[float] = None) -> None:
        """``det notebook|shell|tensorboard|command set priority`` / ``det job update``."""
        with self.lock:
            row = self.db.one("SELECT config FROM tasks WHERE id=?", [task_id])
            cfg = dict((row or {}).get("config") or {})
            if priority is not None:
                cfg["priority"] = int(priority)
                self.sched.set_priority(task_id, int(priority))
            if weight is not None:
                cfg["weight"] = float(weight)
                self.sched.set_weight(task_id, float(weight))
            self.db.update("tasks", "id", task_id, config=cfg)
            self.cv.notify_all()

    # ================================================================ resource pools
    def check_pool(self, name: Optional[str], slots: int, workspace: Optional[str]) -> str:
        """The pool a request lands in (named, or the compute / aux default by slots); a pool bound
        to workspaces takes only their experiments (reference ``api_resourcepool.go`` bindings)."""
        from determined_amd.master._pools import PoolError

        try:
            pool = self.sched.resolve(name, slots)
        except PoolError as e:
            raise ValueError(str(e))
        if workspace is not None:
            bound = self.pool_bindings(pool)
            if bound:
                w = self.db.one("SELECT id FROM workspaces WHERE name=?", [workspace])
                if w is None or int(w["id"]) not in bound:
                    raise ValueError(f"resource pool {pool!r} is bound to other workspaces than {workspace!r}")
        return pool

    def allocation_usage(self, after: float, before: float) -> List[Dict[str, Any]]:
        """Allocations that held slots in [after, before), with the overlap in seconds."""
        now = time.time()
        rows = self.db.all("SELECT * FROM allocation_history WHERE start_time < ? AND (end_time IS NULL OR end_time > ?) "
                           "ORDER BY start_time", [before, after])
        for r in rows:
            end = r["end_time"] if r["end_time"] is not None else now
            r["seconds"] = max(0.0, min(end, before) - max(r["start_time"], after))
            r["slot_seconds"] = r["seconds"] * int(r["slots"] or 0)
        return rows

    def pool_bindings(self, pool: str) -> List[int]:
        return [int(r["workspace_id"]) for r in self.db.all("SELECT workspace_id FROM pool_bindings WHERE pool=? "
                                                             "ORDER BY workspace_id", [pool])]

    def set_pool_bindings(self, pool: str, workspace_ids: List[int], mode: str) -> List[int]:
        """``mode``: add / remove / replace the workspaces bound to ``pool``."""
        if pool not in self.sched.pools:
            raise KeyError(f"resource pool {pool!r} does not exist")
        with self.lock:
            cur = set(self.pool_bindings(pool))
            ids = {int(w) for w in workspace_ids}
            new = cur | ids if mode == "add" else (cur - ids if mode == "remove" else ids)
            self.db.execute("DELETE FROM pool_bindings WHERE pool=?", [pool])
            for w in sorted(new):
                self.db.execute("INSERT INTO pool_bindings (pool, workspace_id) VALUES (?, ?)", [pool, w])
            return sorted(new)

    def pools_for_workspace(self, workspace_id: int) -> List[str]:
        """Pools a workspace's experiments may use: unbound pools + the ones bound to it."""
        return [p for p in self.sched.pools if not self.pool_bindings(p) or int(workspace_id) in self.pool_bindings(p)]

    def _drop_allocation(self, a: Allocation) -> None:
        self.sched.remove_request(a.id)
        a.state = "TERMINATED"
        if a.exp_id is not None and a.exp_id in self.experiments:
            exp = self.experiments[a.exp_id]
            if exp.deferred:
                self._drain_deferred(exp)
        self.cv.notify_all()

    # ================================================================ experiment settings
    def set_experiment_resources(self, eid: int, max_slots: Any = "unset", weight: Optional[float] = None,
                                 priority: Optional[int] = None) -> None:
        """``det experiment set max-slots|weight|priority`` / job-queue updates."""
        with self.lock:
            exp = self._exp(eid)
            res = exp.config.setdefault("resources", {})
            if max_slots != "unset":
                res["max_slots"] = None if max_slots is None else int(max_slots)
                self.sched.set_max_slots(f"exp-{eid}", res["max_slots"])
            if weight is not None:
                res["weight"] = float(weight)
                self.sched.set_weight(f"exp-{eid}", float(weight))
            if priority is not None:
                res["priority"] = int(priority)
                self.sched.set_priority(f"exp-{eid}", int(priority))
            self.db.update("experiments", "id", eid, config=exp.config)
            self._drain_deferred(exp)
            self.cv.notify_all()

    def patch_experiment_config(self, eid: int, section: str, values: Dict[str, Any]) -> Dict[str, Any]:
        """Update a mutable config section (checkpoint_storage GC policy, retention_policy)."""
        if section not in ("checkpoint_storage", "retention_policy"):
            raise ValueError(f"config section {section!r} is not mutable")
        with self.lock:
            row = self.db.one("SELECT config FROM experiments WHERE id=?", [eid])
            if row is None:
                raise KeyError(f"experiment {eid} not found")
            cfg = row["config"]
            sec = dict(cfg.get(section) or {})
            sec.update(values)
            cfg[section] = sec
            self.db.update("experiments", "id", eid, config=cfg)
            if eid in self.experiments:
                self.experiments[eid].config = cfg
            return cfg

    def continue_experiment(self, eid: int, overrides: Optional[Dict[str, Any]] = None) -> int:
        """``det experiment continue``: a new single-trial experiment warm-started from the
        parent's latest (or best) checkpoint, same model definition."""
        import copy

        row = self.db.one("SELECT * FROM experiments WHERE id=?", [eid])
        if row is None:
            raise KeyError(f"experiment {eid} not found")
        trials = self.db.all("SELECT id, hparams, latest_checkpoint FROM trials WHERE experiment_id=? ORDER BY id",
                             [eid])
        if len(trials) != 1:
            raise ValueError("continue needs an experiment with exactly one trial")
        ck = trials[0]["latest_checkpoint"]
        cfg = copy.deepcopy(row["config"])
        for k, v in (overrides or {}).items():
            cur = cfg
            parts = k.split(".")
            for p in parts[:-1]:
                cur = cur.setdefault(p, {})
            cur[parts[-1]] = v
        hp = trials[0]["hparams"] or {}
        cfg["hyperparameters"] = {k: {"type": "const", "val": v} for k, v in hp.items()}
        cfg["searcher"] = dict(cfg["searcher"], name="single", source_checkpoint_uuid=ck)
        for k in ("max_trials", "max_concurrent_trials", "mode", "divisor", "max_rungs"):
            cfg["searcher"].pop(k, None)
        return self.create_experiment(cfg, row["model_def"], parent_id=eid)

    def _kill_allocation(self, a: Allocation) -> None:
        a.killed = True
        if a.state == "PENDING":
            self._drop_allocation(a)
            self._on_allocation_exit(a)
            return
        for agent_id, _ in a.assignment:
            ag = self.agents.get(agent_id)
            if ag is not None:
                ag["queue"].append({"type": "kill", "allocation_id": a.id})
        a.state = "TERMINATING"
        self.cv.notify_all()

    def pause_task(self, task_id: str) -> None:
        """``det task pause`` (reference ``api_generic_tasks.go`` PauseGenericTask): end the
        task's allocation and park the task in PAUSED; ``unpause_task`` starts it again with the
        same command, environment and resources."""
        with self.lock:
            row = self.db.one("SELECT * FROM tasks WHERE id=?", [task_id])
            if row is None:
                raise KeyError(f"task {task_id} not found")
            if row["state"] in ("TERMINATED", "CANCELED", "PAUSED", "ERROR", "COMPLETED"):
                raise ValueError(f"cannot pause task {task_id} in state {row['state']}")
            live = [a for a in self.allocations.values() if a.task_id == task_id and a.state != "TERMINATED"]
            for a in live:
                a.pausing = True  # type: ignore[attr-defined]
                self._kill_allocation(a)
            if not live:
                self.db.update("tasks", "id", task_id, state="PAUSED")
            self.cv.notify_all()

    def unpause_task(self, task_id: str) -> None:
        with self.lock:
            row = self.db.one("SELECT * FROM tasks WHERE id=?", [task_id])
            if row is None:
                raise KeyError(f"task {task_id} not found")
            if row["state"] != "PAUSED":
                raise ValueError(f"task {task_id} is not paused (state {row['state']})")
            prev = [a for a in self.allocations.values() if a.task_id == task_id]
            cfg = row.get("config") or {}
            n = 1 + sum(1 for _ in prev)
            aid = f"{task_id}.{n}"
            a = Allocation(aid, task_id, int(cfg.get("slots", 0)), kind=row["type"])
            last = prev[-1] if prev else None
            a.command = cfg.get("cmd")  # type: ignore[attr-defined]
            a.env = getattr(last, "env", {}) if last is not None else {}  # type: ignore[attr-defined]
            a.task_config = getattr(last, "task_config", None) if last is not None else None  # type: ignore
            a.workdir_b64 = getattr(last, "workdir_b64", None) if last is not None else None  # type: ignore[attr-defined]
            self.allocations[aid] = a
            self.db.update("tasks", "id", task_id, state="PENDING", end_time=None, exit_code=None)
            self.sched.add_request(aid, task_id, a.slots, int(cfg.get("priority", 42)), float(cfg.get("weight", 1.0)),
                                   self._next_order(), False, pool=cfg.get("resource_pool"))
            self.cv.notify_all()

    def kill_task(self, task_id: str) -> None:
        with self.lock:
            for a in list(self.allocations.values()):
                if a.task_id == task_id and a.state != "TERMINATED":
                    self._kill_allocation(a)

    def _schedule(self) -> None:
        d = self.sched.schedule()
        reqs = None
        for aid in d["allocated"]:
            a = self.allocations.get(aid)
            if a is None:
                continue
            reqs = reqs or self.sched.requests()
            a.assignment = [(ag, list(sl)) for ag, sl in reqs[aid]["assignment"]]
            a.state = "ASSIGNED"
            self._record_allocation_start(a, reqs[aid].get("resource_pool"))
            self._dispatch(a)
        for aid in d["preempt"]:
            a = self.allocations.get(aid)
            if a is not None:
                a.preempt = True
        if d["allocated"] or d["preempt"]:
            self.cv.notify_all()

    def _dispatch(self, a: Allocation) -> None:
        hosts = [self.agents[ag]["host"] for ag, _ in a.assignment]
        for rank, (agent_id, slots) in enumerate(a.assignment):
            ag = self.agents[agent_id]
            devices = [ag["devices"][s] for s in slots] if ag.get("devices") else slots
            env = {
                "DET_MASTER": self.master_url,
                "DET_CLUSTER_ID": self.cluster_id,
                "DET_AGENT_ID": agent_id,
                "DET_AGENT_HOST": ag.get("host", "127.0.0.1"),
                "DET_ALLOCATION_ID": a.id,
                "DET_TASK_ID": a.task_id,
                "DET_SESSION_TOKEN": self.auth_token or "",
                "DET_SLOT_IDS": json.dumps(devices),
                "DET_CONTAINER_ADDRS": json.dumps(hosts),
                "DET_CONTAINER_RANK": str(rank),
                "DET_TASK_TYPE": a.kind,
                "DET_USE_GPU": "1" if ag.get("gpu") else "0",
            }
            cmd: Dict[str, Any] = {"type": "start", "allocation_id": a.id, "task_id": a.task_id, "devices": devices,
                                   "gpu": bool(ag.get("gpu")), "env": env}
            if a.kind == "TRIAL":
                exp = self.experiments[a.exp_id]  # type: ignore[index]
                tr = next(t for t in exp.trials.values() if t.id == a.trial_id)
                tr.run_id += 1
                cfg = exp.config
                env.update({
                    "DET_TRIAL_ID": str(tr.id),
                    "DET_EXPERIMENT_ID": str(exp.id),
                    "DET_TRIAL_SEED": str(tr.seed),
                    "DET_HPARAMS": json.dumps(tr.hparams),
                    "DET_EXPERIMENT_CONFIG": json.dumps(cfg),
                    "DET_STEPS_COMPLETED": str(tr.total_batches),
                    "DET_TRIAL_RUN_ID": str(tr.run_id),
                    "DET_LATEST_CHECKPOINT": tr.latest_checkpoint or tr.warm_start or "",
                })
                for kv in _env_list(cfg.get("environment", {}).get("environment_variables")):
                    k, _, v = kv.partition("=")
                    env[k] = v
                env.update(self._agent_user_env(a.exp_id))
                cmd.update(entrypoint=cfg.get("entrypoint"), slots_per_trial=a.slots,
                           model_def_url=f"/api/v1/experiments/{exp.id}/model_def")
                self._persist_trial(tr)
            else:
                cmd.update(command=getattr(a, "command", []), workdir_b64=getattr(a, "workdir_b64", None))
                env.update(getattr(a, "env", {}))
                if getattr(a, "task_config", None):
                    env["DET_TASK_CONFIG"] = json.dumps(a.task_config)
                self.db.update("tasks", "id", a.task_id, state="RUNNING")
            ag["queue"].append(cmd)
        self.cv.notify_all()

    # ================================================================ agents
    def register_agent(self, agent_id: str, slots: int, host: str = "127.0.0.1", devices: Optional[List[Any]] = None,
                       gpu: bool = False, label: str = "", resource_pool: Optional[str] = None,
                       running: Optional[List[str]] = None) -> Dict[str, Any]:
        with self.lock:
            existing = self.agents.get(agent_id)
            if existing is not None and running is not None:
                # a re-registering agent lists what it still runs: allocations it was given and no
                # longer knows (its process restarted) are lost, like a lost agent's (reference
                # test_agent_restart: without container reattach the trial restarts)
                # ASSIGNED counts too: an agent that pulled a start from its queue and died before
                # reporting 'started' no longer has it (the agent lists allocations from the moment it
                # receives their start command)
                alive = set(running)
                queued = {c.get("allocation_id") for c in existing.get("queue", []) if c.get("type") == "start"}
                for a in list(self.allocations.values()):
                    if a.state in ("ASSIGNED", "RUNNING") and a.id not in alive and a.id not in queued and \
                            any(x[0] == agent_id for x in a.assignment):
                        logger.warning(f"agent {agent_id} restarted without allocation {a.id}: marking it lost")
                        a.exit_codes[agent_id] = -1
                        self._finish_allocation(a)
            pool = resource_pool or (existing or {}).get("resource_pool") or self.sched.default_compute
            if pool not in self.sched.pools:
                raise ValueError(f"resource pool {pool!r} does not exist (pools: {sorted(self.sched.pools)})")
            if existing is not None and (pool != existing.get("resource_pool") or slots != existing.get("slots")):
                # moved to another pool / changed its slot count: the scheduler entry is rebuilt, and the
                # allocations placed through the old entry are lost (their trials restart under
                # max_restarts in the new layout) instead of being accounted in the wrong pool
                logger.warning(f"agent {agent_id} re-registered with pool {pool!r} / {slots} slots (was "
                               f"{existing.get('resource_pool')!r} / {existing.get('slots')}): rebuilding it")
                for a in list(self.allocations.values()):
                    if a.state in ("ASSIGNED", "RUNNING") and any(x[0] == agent_id for x in a.assignment):
                        a.exit_codes[agent_id] = -1
                        self._finish_allocation(a)
                existing["queue"] = [c for c in existing.get("queue", []) if c.get("type") != "start"]
                self.sched.remove_agent(agent_id)
                self.sched.add_agent(agent_id, slots, pool)
            self.agents[agent_id] = {"id": agent_id, "slots": slots, "host": host, "devices": devices or list(range(slots)),
                                     "gpu": gpu, "label": label, "queue": existing["queue"] if existing else [],
                                     "last_seen": time.time(), "enabled": existing["enabled"] if existing else True,
                                     "resource_pool": pool,
                                     "disabled_slots": list((existing or {}).get("disabled_slots") or [])}
            if existing is None:
                self.sched.add_agent(agent_id, slots, pool)
            self.cv.notify_all()
            return {"cluster_id": self.cluster_id}

    def agent_poll(self, agent_id: str, timeout: float) -> List[Dict[str, Any]]:
        deadline = time.time() + timeout
        with self.lock:
            ag = self.agents.get(agent_id)
            if ag is None:
                raise KeyError(f"agent {agent_id} not registered")
            while not ag["queue"] and time.time() < deadline and not self._closed:
                ag["last_seen"] = time.time()
                self.cv.wait(max(0.0, min(1.0, deadline - time.time())))
            ag["last_seen"] = time.time()
            out, ag["queue"] = ag["queue"], []
            return out

    def _check_agents(self, stale_s: float = 120.0) -> None:
        now = time.time()
        for aid, ag in list(self.agents.items()):
            if now - ag["last_seen"] > stale_s:
                logger.warning(f"agent {aid} lost")
                self.sched.remove_agent(aid)
                del self.agents[aid]
                for a in list(self.allocations.values()):
                    if any(x[0] == aid for x in a.assignment) and a.state in ("ASSIGNED", "RUNNING"):
                        a.exit_codes[aid] = -1
                        self._finish_allocation(a)

    def agent_event(self, agent_id: str, ev: Dict[str, Any]) -> None:
        with self.lock:
            a = self.allocations.get(ev["allocation_id"])
            if a is None:
                return
            if ev["type"] == "started":
                a.state = "RUNNING"
                if a.kind != "TRIAL":
                    pass
            elif ev["type"] == "exited":
                a.exit_codes[agent_id] = int(ev.get("exit_code", -1))
                if len(a.exit_codes) >= len(a.assignment):
                    self._finish_allocation(a)
            self.cv.notify_all()

    def _agent_user_env(self, exp_id: Optional[int]) -> Dict[str, str]:
        """The experiment owner's linked agent user/group (``det user link-with-agent-user``)."""
        row = self.db.one("SELECT u.agent_uid, u.agent_gid, u.agent_user, u.agent_group FROM experiments e "
                          "JOIN users u ON u.username = e.owner WHERE e.id=?", [exp_id]) if exp_id is not None else None
        out: Dict[str, str] = {}
        for col, key in (("agent_uid", "DET_AGENT_UID"), ("agent_gid", "DET_AGENT_GID"),
                         ("agent_user", "DET_AGENT_USER"), ("agent_group", "DET_AGENT_GROUP")):
            if row is not None and row.get(col) is not None:
                out[key] = str(row[col])
        return out

    def _record_allocation_start(self, a: Allocation, pool: Optional[str]) -> None:
        """Slot usage history (``det resources raw|aggregated``; reference
        ``master/internal/db/postgres_resourcemanagers`` allocation accounting)."""
        owner = None
        if a.exp_id is not None and a.exp_id in self.experiments:
            row = self.db.one("SELECT owner FROM experiments WHERE id=?", [a.exp_id])
            owner = row["owner"] if row else None
        self.db.execute("INSERT OR REPLACE INTO allocation_history (alloc_id, task_id, kind, experiment_id, owner, "
                        "resource_pool, slots, start_time, end_time) VALUES (?, ?, ?, ?, ?, ?, ?, ?, NULL)",
                        [a.id, a.task_id, a.kind, a.exp_id, owner, pool, a.slots, time.time()])

    def _finish_allocation(self, a: Allocation) -> None:
        if a.state == "TERMINATED":
            return
        self.db.execute("UPDATE allocation_history SET end_time=? WHERE alloc_id=? AND end_time IS NULL",
                        [time.time(), a.id])
        self.sched.remove_request(a.id)
        a.state = "TERMINATED"
        self._on_allocation_exit(a)
        if a.exp_id is not None and a.exp_id in self.experiments and self.experiments[a.exp_id].deferred:
            self._drain_deferred(self.experiments[a.exp_id])
        self.cv.notify_all()

    def _on_allocation_exit(self, a: Allocation) -> None:
        ok = all(c == 0 for c in a.exit_codes.values()) and bool(a.exit_codes)
        if a.kind != "TRIAL":
            code = max(a.exit_codes.values()) if a.exit_codes else -1
            state = "TERMINATED" if not a.killed else "CANCELED"
            if getattr(a, "pausing", False):
                state = "PAUSED"  # det task pause: the allocation ended, the task waits for unpause
            self.db.update("tasks", "id", a.task_id, state=state, end_time=time.time(), exit_code=code)
            return
        exp = self.experiments.get(a.exp_id)  # type: ignore[arg-type]
        if exp is None:
            return
        try:
            _, tr = self._trial(a.trial_id)  # type: ignore[arg-type]
        except KeyError:
            return
        tr.allocation = None
        ops: List[Dict[str, Any]] = []
        if a.killed or exp.state in ("STOPPING_CANCELED", "STOPPING_ERROR"):
            ops = self._finish_trial(exp, tr, "CANCELED")
        elif tr.early_exit:
            ops = self._finish_trial(exp, tr, "COMPLETED")
        elif (ok and not a.preempt and tr.ops and
              getattr(a, "progress_at_start", None) == (tr.total_batches, len(tr.ops))):
            # a clean exit that trained nothing and completed no searcher operation, without being
            # preempted: counted as a failed run (max_restarts) instead of being rescheduled forever
            tr.restarts += 1
            max_restarts = int(exp.config.get("max_restarts", 5))
            logger.warning(f"trial {tr.id} exited cleanly without progress; restart {tr.restarts}/{max_restarts}")
            if tr.restarts > max_restarts or tr.no_retry:
                ops = self._finish_trial(exp, tr, "ERROR")
            elif exp.state == "ACTIVE":
                self._request_allocation(exp, tr)
        elif ok or (a.preempt and a.ack_preempt):
            if tr.close_requested and not tr.ops:
                ops = self._finish_trial(exp, tr, "COMPLETED")
            elif tr.ops and exp.state == "ACTIVE":
                self._request_allocation(exp, tr)
            # else: waiting for the searcher (e.g. an ASHA promotion) or paused
        else:
            tr.restarts += 1
            max_restarts = int(exp.config.get("max_restarts", 5))
            logger.warning(f"trial {tr.id} failed (exit {a.exit_codes}); restart {tr.restarts}/{max_restarts}")
            if tr.restarts > max_restarts or tr.no_retry:
                ops = self._finish_trial(exp, tr, "ERROR")
            elif exp.state == "ACTIVE":
                self._request_allocation(exp, tr)
        self._persist_trial(tr)
        self._process_ops(exp, ops)

    # ================================================================ harness-facing
    def get_searcher_op(self, tid: int) -> Dict[str, Any]:
        with self.lock:
            _, tr = self._trial(tid)
            if tr.ops:
                return {"completed": False, "op": {"validate_after": {"length": tr.ops[0]}}}
            return {"completed": True, "op": None}

    def complete_searcher_op(self, tid: int, length: int, metric: Any) -> None:
        with self.lock:
            exp, tr = self._trial(tid)
            if not tr.ops or tr.ops[0] != int(length):
                raise ValueError(f"trial {tid} has no pending operation of length {length} (pending {tr.ops})")
            tr.ops.pop(0)
            self.db.update("trials", "id", tid, searcher_metric=float(metric) if _isnum(metric) else None)
            self._persist_trial(tr)
            if exp.searcher is not None:
                ops = exp.searcher.validation_completed(tr.request_id, float(metric), int(length))
                self._process_ops(exp, ops)
            else:
                self._custom_event(exp, {"validation_completed": {"request_id": tr.request_id, "metric": metric,
                                                                  "validate_after_length": int(length)}})
            self.cv.notify_all()

    def report_progress(self, tid: int, progress: float) -> None:
        with self.lock:
            exp, tr = self._trial(tid)
            if exp.searcher is not None:
                exp.searcher.set_trial_progress(tr.request_id, progress)
                exp.progress = exp.searcher.progress()
                self.db.update("experiments", "id", exp.id, progress=exp.progress)

    def report_metrics(self, tid: int, body: Dict[str, Any]) -> None:
        with self.lock:
            group = body["group"]
            self.db.insert("metrics", trial_id=tid, trial_run_id=body.get("trial_run_id", 0), group_name=group,
                           steps_completed=int(body["steps_completed"]), metrics=body["metrics"],
                           batch_metrics=body.get("batch_metrics"), ts=time.time())
            if group in ("training", "validation"):
                try:
                    exp, tr = self._trial(tid)
                    tr.total_batches = max(tr.total_batches, int(body["steps_completed"]))
                    self._persist_trial(tr)
                    if group == "validation":
                        m = exp.config["searcher"].get("metric")
                        v = body["metrics"].get(m)
                        if _isnum(v):
                            row = self.db.one("SELECT best_validation FROM trials WHERE id=?", [tid])
                            sib = exp.config["searcher"].get("smaller_is_better", True)
                            best = row["best_validation"] if row else None
                            if best is None or (v < best if sib else v > best):
                                self.db.update("trials", "id", tid, best_validation=float(v))
                except KeyError:
                    pass

    def report_checkpoint(self, body: Dict[str, Any]) -> None:
        with self.lock:
            tid = body.get("trial_id")
            exp_id = None
            metric = None
            steps = body.get("steps_completed") or (body.get("metadata") or {}).get("steps_completed")
            if tid is not None:
                try:
                    exp, tr = self._trial(int(tid))
                    exp_id = exp.id
                    tr.latest_checkpoint = body["uuid"]
                    if steps is not None:
                        tr.total_batches = max(tr.total_batches, int(steps))
                    self._persist_trial(tr)
                    m = exp.config["searcher"].get("metric")
                    row = self.db.one("SELECT metrics FROM metrics WHERE trial_id=? AND group_name='validation' "
                                      "AND steps_completed=? ORDER BY id DESC", [tid, steps])
                    if row and _isnum((row["metrics"] or {}).get(m)):
                        metric = float(row["metrics"][m])
                except KeyError:
                    row = self.db.one("SELECT experiment_id FROM trials WHERE id=?", [tid])
                    exp_id = row["experiment_id"] if row else None
            self.db.execute("INSERT OR REPLACE INTO checkpoints (uuid, trial_id, experiment_id, task_id, allocation_id,"
                            " state, resources, metadata, steps_completed, report_time, searcher_metric) VALUES "
                            "(?,?,?,?,?,?,?,?,?,?,?)",
                            [body["uuid"], tid, exp_id, body.get("task_id"), body.get("allocation_id"), "COMPLETED",
                             json.dumps(body.get("resources") or {}), json.dumps(body.get("metadata") or {}),
                             steps, time.time(), metric])

    def early_exit(self, tid: int, reason: str) -> None:
        with self.lock:
            exp, tr = self._trial(tid)
            if tr.early_exit is not None:
                raise ValueError("early exit already reported")
            tr.early_exit = {"EXITED_REASON_INVALID_HP": "invalid_hp",
                             "EXITED_REASON_USER_REQUESTED_STOP": "user_requested_stop"}.get(reason, "errored")
            self._persist_trial(tr)

    def preemption_signal(self, alloc_id: str, timeout: float) -> bool:
        deadline = time.time() + timeout
        with self.lock:
            a = self.allocations.get(alloc_id)
            if a is None:
                return True
            while not a.preempt and time.time() < deadline and not self._closed:
                self.cv.wait(max(0.0, min(1.0, deadline - time.time())))
            return a.preempt

    def allocation_all_gather(self, alloc_id: str, request_uuid: str, num_peers: int, data: Any,
                              rank: Optional[int] = None, timeout: float = 600.0) -> List[Any]:
        """Block until ``num_peers`` processes of the allocation have posted, then return every
        peer's ``data`` (ordered by ``rank`` when given, else by arrival).  Containers use it to
        exchange addresses when the launcher cannot know them up front (Kubernetes pods);
        reference ``master/internal/task/allgather``."""
        deadline = time.time() + timeout
        with self.lock:
            a = self.allocations.get(alloc_id)
            if a is None:
                raise KeyError(f"allocation {alloc_id} not found")
            for res, members in a.gather_done.values():
                if request_uuid in members:  # a retried post of a finished round (lost response)
                    return list(res)
            my_round = a.gather_round
            a.gather[request_uuid] = (rank if rank is not None else len(a.gather), data)
            if len(a.gather) >= num_peers:
                res = [d for _, d in sorted(a.gather.values(), key=lambda kv: kv[0])]
                a.gather_done[my_round] = (res, frozenset(a.gather))
                a.gather_done.pop(my_round - 4, None)  # keep the last few rounds for late re-fetches
                a.gather, a.gather_round = {}, my_round + 1
                self.cv.notify_all()
            while my_round not in a.gather_done and time.time() < deadline and not self._closed:
                if a.state == "TERMINATED":
                    raise RuntimeError(f"allocation {alloc_id} terminated during all-gather")
                self.cv.wait(max(0.0, min(1.0, deadline - time.time())))
            if my_round not in a.gather_done:
                if a.gather_round == my_round:
                    a.gather.pop(request_uuid, None)
                raise TimeoutError(f"all-gather of allocation {alloc_id} timed out")
            return list(a.gather_done[my_round][0])

    def ack_preemption(self, alloc_id: str) -> None:
        with self.lock:
            a = self.allocations.get(alloc_id)
            if a is not None:
                a.ack_preempt = True

    def best_searcher_validation(self, eid: int) -> Optional[float]:
        with self.lock:
            exp = self._exp(eid)
            sib = exp.config["searcher"].get("smaller_is_better", True)
            row = self.db.one(f"SELECT {'MIN' if sib else 'MAX'}(best_validation) AS v FROM trials WHERE experiment_id=?",
                              [eid])
            return row["v"] if row else None

    # ================================================================ logs
    def add_logs(self, task_id: str, logs: List[Dict[str, Any]], allocation_id: Optional[str] = None) -> None:
        with self.lock:
            now = time.time()
            self.db.conn.executemany(
                "INSERT INTO task_logs (task_id, allocation_id, rank, ts, log) VALUES (?,?,?,?,?)",
                [(task_id, allocation_id, l.get("rank"), now, l["log"]) for l in logs])
            self._apply_log_policies(task_id, allocation_id, logs)
            self._log_webhooks(task_id, logs)
            self.cv.notify_all()

    def _log_webhooks(self, task_id: str, logs: List[Dict[str, Any]]) -> None:
        if not task_id.startswith("trial-"):
            return
        hooks = self.db.all("SELECT triggers FROM webhooks")
        rxs = [t["condition"]["regex"] for h in hooks for t in (h.get("triggers") or [])
               if isinstance(t, dict) and t.get("trigger_type") == "TASK_LOG" and (t.get("condition") or {}).get("regex")]
        if not rxs:
            return
        try:
            exp, tr = self._trial(int(task_id.split("-", 1)[1]))
        except (KeyError, ValueError):
            return
        for l in logs:
            if any(re.search(rx, l.get("log", "")) for rx in rxs):
                self._fire_webhooks(exp, "TASK_LOG", tr, log_line=l.get("log", ""))

    def _apply_log_policies(self, task_id: str, allocation_id: Optional[str], logs: List[Dict[str, Any]]) -> None:
        """Experiment ``log_policies`` (reference ``master/internal/logpattern``): a regex match in a
        trial's logs can cancel its remaining restarts (``cancel_retries``) or keep its next
        allocations off the agent that produced the line (``exclude_node``)."""
        if not task_id.startswith("trial-"):
            return
        try:
            exp, tr = self._trial(int(task_id.split("-", 1)[1]))
        except (KeyError, ValueError):
            return
        policies = exp.config.get("log_policies") or []
        if not policies:
            return
        import re

        a = self.allocations.get(allocation_id) if allocation_id else tr.allocation
        for pol in policies:
            try:
                rx = re.compile(pol["pattern"])
            except (re.error, KeyError, TypeError):
                continue
            if not any(rx.search(l.get("log", "")) for l in logs):
                continue
            act = (pol.get("action") or {}).get("type")
            if act == "cancel_retries" and not tr.no_retry:
                tr.no_retry = True
                logger.info(f"trial {tr.id}: log policy {pol['pattern']!r} matched; retries cancelled")
            elif act == "exclude_node" and a is not None:
                for agent_id, _ in a.assignment:
                    if agent_id not in tr.excluded_agents:
                        tr.excluded_agents.append(agent_id)
                        logger.info(f"trial {tr.id}: log policy {pol['pattern']!r} matched; excluding {agent_id}")

    def cleanup_logs(self, now: Optional[float] = None) -> int:
        """Log retention (``retention_policy.log_retention_days``, experiment config or master
        default ``DET_LOG_RETENTION_DAYS``): delete logs of trials that ended longer ago."""
        now = time.time() if now is None else now
        deleted = 0
        default_days = os.environ.get("DET_LOG_RETENTION_DAYS")
        with self.lock:
            for row in self.db.all("SELECT id, config FROM experiments"):
                days = ((row["config"] or {}).get("retention_policy") or {}).get("log_retention_days")
                if days is None and default_days is not None:
                    days = int(default_days)
                if days is None or int(days) < 0:
                    continue
                cutoff = now - int(days) * 86400
                for t in self.db.all("SELECT id FROM trials WHERE experiment_id=? AND end_time IS NOT NULL AND "
                                     "end_time < ? AND log_retention_days IS NULL", [row["id"], cutoff]):
                    cur = self.db.execute("DELETE FROM task_logs WHERE task_id=?", [f"trial-{t['id']}"])
                    deleted += cur.rowcount or 0
            # per-trial overrides (``det trial set log-retention``; -1 keeps forever)
            for t in self.db.all("SELECT id, end_time, log_retention_days FROM trials WHERE "
                                 "log_retention_days IS NOT NULL AND log_retention_days >= 0 AND end_time IS NOT NULL"):
                if t["end_time"] < now - int(t["log_retention_days"]) * 86400:
                    cur = self.db.execute("DELETE FROM task_logs WHERE task_id=?", [f"trial-{t['id']}"])
                    deleted += cur.rowcount or 0
        return deleted

    def get_logs(self, task_id: str, after_id: int = 0, limit: int = 10000) -> List[Dict[str, Any]]:
        return self.db.all("SELECT id, rank, ts, log FROM task_logs WHERE task_id=? AND id>? ORDER BY id LIMIT ?",
                           [task_id, after_id, limit])

    # ================================================================ custom searcher
    def _custom_event(self, exp: ExperimentRec, ev: Dict[str, Any]) -> None:
        if exp.searcher is not None:
            return
        exp.custom_event_id += 1
        ev = dict(ev)
        ev["id"] = exp.custom_event_id
        exp.custom_events.append(ev)
        self.cv.notify_all()

    def get_searcher_events(self, eid: int, timeout: float = 0) -> List[Dict[str, Any]]:
        deadline = time.time() + timeout
        with self.lock:
            exp = self._exp(eid)
            while not exp.custom_events and time.time() < deadline and exp.state not in TERMINAL_EXP:
                self.cv.wait(max(0.0, min(1.0, deadline - time.time())))
            return list(exp.custom_events)

    def post_searcher_operations(self, eid: int, ops: List[Dict[str, Any]], triggered_by_event: int) -> None:
        with self.lock:
            exp = self._exp(eid)
            exp.custom_events = [e for e in exp.custom_events if e["id"] > triggered_by_event]
            self._process_ops(exp, ops)
            self.cv.notify_all()

    # ================================================================ checkpoint GC
    def gc_experiment_checkpoints(self, eid: int, delete_all: bool = False) -> List[str]:
        """Keep save_trial_latest / save_trial_best per trial and save_experiment_best overall
        (reference ``master/internal/checkpoint_gc.go`` + ``exec/gc_checkpoints.py``)."""
        from determined_amd import storage

        with self.lock:
            row = self.db.one("SELECT config FROM experiments WHERE id=?", [eid])
            if row is None:
                return []
            cfg = row["config"]
            cs = cfg["checkpoint_storage"]
            sib = cfg["searcher"].get("smaller_is_better", True)
            ckpts = self.db.all("SELECT uuid, trial_id, steps_completed, searcher_metric FROM checkpoints WHERE "
                                "experiment_id=? AND state='COMPLETED'", [eid])
            keep = set()
            if not delete_all:
                by_trial: Dict[int, List[Dict[str, Any]]] = {}
                for c in ckpts:
                    by_trial.setdefault(c["trial_id"], []).append(c)

                def key(c: Dict[str, Any]) -> float:
                    m = c["searcher_metric"]
                    return float("inf") if m is None else (m if sib else -m)

                for cs_list in by_trial.values():
                    latest = sorted(cs_list, key=lambda c: -(c["steps_completed"] or 0))
                    keep.update(c["uuid"] for c in latest[: int(cs.get("save_trial_latest", 1))])
                    keep.update(c["uuid"] for c in sorted(cs_list, key=key)[: int(cs.get("save_trial_best", 1))]
                                if c["searcher_metric"] is not None)
                    # the latest checkpoint of a still-running trial is always kept (needed to resume)
                keep.update(c["uuid"] for c in sorted(ckpts, key=key)[: int(cs.get("save_experiment_best", 0))]
                            if c["searcher_metric"] is not None)
                for tr in self.experiments.get(eid, ExperimentRec(eid, cfg, "")).trials.values():
                    if tr.latest_checkpoint and tr.state not in TERMINAL_TRIAL:
                        keep.add(tr.latest_checkpoint)
            doomed = [c["uuid"] for c in ckpts if c["uuid"] not in keep]
            if cfg.get("checkpoint_policy") == "none" and not delete_all:
                doomed = [c["uuid"] for c in ckpts]
        try:
            sm = storage.build(cs)
        except Exception as e:
            logger.warning(f"checkpoint GC skipped: {e}")
            return []
        for u in doomed:
            try:
                sm.delete(u)
            except Exception as e:
                logger.warning(f"failed to delete checkpoint {u}: {e}")
            self.db.update("checkpoints", "uuid", u, state="DELETED")
        return doomed

    def delete_checkpoints(self, uuids: List[str]) -> None:
        from determined_amd import storage

        for u in uuids:
            row = self.db.one("SELECT c.uuid, e.config FROM checkpoints c LEFT JOIN experiments e "
                              "ON c.experiment_id=e.id WHERE c.uuid=?", [u])
            if row is None:
                continue
            if row.get("config"):
                try:
                    storage.build(row["config"]["checkpoint_storage"]).delete(u)
                except Exception as e:
                    logger.warning(f"delete {u}: {e}")
            self.db.update("checkpoints", "uuid", u, state="DELETED")

    # ================================================================ webhooks
    def _fire_webhooks(self, exp: ExperimentRec, trigger: str, trial: Optional[TrialRec] = None,
                       log_line: Optional[str] = None) -> None:
        """POST an event to every matching webhook (reference ``master/internal/webhooks``).

        Triggers: ``EXPERIMENT_STATE_CHANGE`` (``condition: {"state": S}`` narrows it) and
        ``TASK_LOG`` (``condition: {"regex": R}`` over trial log lines).  ``webhook_type``
        ``SLACK`` posts a Slack ``{"blocks": ...}`` message, ``DEFAULT`` the JSON event.  Every
        request is signed: ``X-Determined-AMD-Signature: sha256=<hmac(timestamp.body)>`` with
        the master's webhook secret (cluster id) and ``X-Determined-AMD-Timestamp``."""
        hooks = self.db.all("SELECT * FROM webhooks")
        if not hooks:
            return
        payload: Dict[str, Any] = {"event_type": trigger, "timestamp": int(time.time()),
                                   "experiment": {"id": exp.id, "state": exp.state, "name": exp.config.get("name"),
                                                  "workspace": exp.config.get("workspace") or "Uncategorized",
                                                  "project": exp.config.get("project") or "Uncategorized"}}
        if trial is not None:
            payload["trial"] = {"id": trial.id, "state": trial.state}
        if log_line is not None:
            payload["log"] = log_line
        targets = []
        for h in hooks:
            for t in h.get("triggers") or [{"trigger_type": "EXPERIMENT_STATE_CHANGE"}]:
                tt = t.get("trigger_type", t) if isinstance(t, dict) else t
                cond = (t.get("condition") or {}) if isinstance(t, dict) else {}
                if tt != trigger:
                    continue
                if trigger == "EXPERIMENT_STATE_CHANGE" and cond.get("state") and cond["state"] != exp.state:
                    continue
                if trigger == "TASK_LOG" and cond.get("regex") and not re.search(cond["regex"], log_line or ""):
                    continue
                targets.append(h)
                break
        if not targets:
            return
        secret = self.cluster_id.encode()

        def send() -> None:
            import hashlib
            import hmac

            import requests

            for h in targets:
                if h.get("webhook_type") == "SLACK":
                    text = f"Experiment {exp.id} ({exp.config.get('name')}): {trigger} -> {exp.state}"
                    if log_line is not None:
                        text += f"\n`{log_line}`"
                    body = json.dumps({"blocks": [{"type": "section", "text": {"type": "mrkdwn", "text": text}}]})
                else:
                    body = json.dumps(payload)
                ts = str(payload["timestamp"])
                sig = hmac.new(secret, (ts + "." + body).encode(), hashlib.sha256).hexdigest()
                try:
                    requests.post(h["url"], data=body, timeout=5, headers={
                        "Content-Type": "application/json", "X-Determined-AMD-Timestamp": ts,
                        "X-Determined-AMD-Signature": f"sha256={sig}"})
                except Exception as e:
                    logger.debug(f"webhook {h['url']} failed: {e}")

        threading.Thread(target=send, daemon=True).start()


def _env_list(v: Any) -> List[str]:
    if v is None:
        return []
    if isinstance(v, dict):
        out: List[str] = []
        for key in ("cpu", "gpu", "rocm"):
            out += v.get(key) or []
        return out
    return list(v)


def _isnum(v: Any) -> bool:
    return isinstance(v, (int, float)) and not isinstance(v, bool)
