"""Resource pools (reference: master config ``resource_pools`` / ``resource_manager``,
``master/internal/rm/agentrm/resource_pool.go``, workspace bindings ``api_resourcepool.go``).

One native scheduler (``_native/scheduler.cpp``) per pool: every pool has its own agents, its own
scheduling policy (priority / fair_share / round_robin), fitting policy and preemption switch,
and its own job queue.  Agents join a pool when they register (``--resource-pool``); trials ask
for one with ``resources.resource_pool`` (default: ``default_compute_resource_pool``), commands /
notebooks / shells / tensorboards with ``resource_pool`` (default: the compute pool for tasks that
need slots, ``default_aux_resource_pool`` for zero-slot tasks).  :class:`PoolSet` keeps the
single-scheduler interface the master was written against (``add_request`` / ``schedule`` /
``requests`` / ``agents`` / slot totals), dispatching each call to the pool that owns the agent or
the request, so an 8-GPU MI355X node can be one pool or be split, e.g. into a 6-slot training pool
and a 2-slot pool for notebooks and evaluation.
"""

from typing import Any, Dict, List, Optional

DEFAULT_POOL = "default"
_POLICIES = ("priority", "fair_share", "round_robin")


class PoolError(ValueError):
    pass


class Pool:
    def __init__(self, native: Any, name: str, policy: str, fit: str, preemption: bool, description: str = "") -> None:
        if policy not in _POLICIES:
            raise PoolError(f"resource pool {name!r}: scheduler type must be one of {_POLICIES}, got {policy!r}")
        self.name = name
        self.policy = policy
        self.fit = fit
        self.preemption = preemption
        self.description = description
        pol = {"priority": native.Policy.PRIORITY, "fair_share": native.Policy.FAIR_SHARE,
               "round_robin": native.Policy.ROUND_ROBIN}[policy]
        self.sched = native.Scheduler(pol, native.Fit.BEST if fit == "best" else native.Fit.WORST, preemption)


def parse_pools(cfg: Optional[List[Dict[str, Any]]], policy: str, fit: str, preemption: bool) -> List[Dict[str, Any]]:
    """Normalise master-config pool entries (``pool_name``, ``description``, ``scheduler: {type,
    fitting_policy, preemption}``) with the master-wide scheduler settings as defaults."""
    out = []
    for p in cfg or [{"pool_name": DEFAULT_POOL}]:
        name = p.get("pool_name") or p.get("name")
        if not name:
            raise PoolError(f"resource pool entry without pool_name: {p!r}")
        sc = p.get("scheduler") or {}
        out.append({"name": str(name), "description": str(p.get("description", "")),
                    "policy": sc.get("type", policy), "fit": sc.get("fitting_policy", fit),
                    "preemption": bool(sc.get("preemption", preemption))})
    if len({p["name"] for p in out}) != len(out):
        raise PoolError("duplicate resource pool names")
    return out


class PoolSet:
    def __init__(self, native: Any, pools: List[Dict[str, Any]], default_compute: Optional[str] = None,
                 default_aux: Optional[str] = None) -> None:
        self.pools: Dict[str, Pool] = {}
        for p in pools:
            self.pools[p["name"]] = Pool(native, p["name"], p["policy"], p["fit"], p["preemption"], p["description"])
        first = next(iter(self.pools))
        self.default_compute = default_compute or (DEFAULT_POOL if DEFAULT_POOL in self.pools else first)
        self.default_aux = default_aux or self.default_compute
        for d in (self.default_compute, self.default_aux):
            if d not in self.pools:
                raise PoolError(f"default resource pool {d!r} is not configured")
        self._agent_pool: Dict[str, str] = {}
        self._req_pool: Dict[str, str] = {}

    # ---------------------------------------------------------------- pools
    def resolve(self, name: Optional[str], slots: int) -> str:
        """The pool a request uses: the named one, else the compute / aux default by slots."""
        if name:
            if name not in self.pools:
                raise PoolError(f"resource pool {name!r} does not exist (pools: {sorted(self.pools)})")
            return name
        return self.default_compute if slots > 0 else self.default_aux

    def pool_of_agent(self, agent_id: str) -> Optional[str]:
        return self._agent_pool.get(agent_id)

    def pool_of_request(self, alloc_id: str) -> Optional[str]:
        return self._req_pool.get(alloc_id)

    # ---------------------------------------------------------------- agents
    def add_agent(self, agent_id: str, slots: int, pool: Optional[str] = None) -> str:
        name = pool or self.default_compute
        if name not in self.pools:
            raise PoolError(f"agent {agent_id}: resource pool {name!r} does not exist (pools: {sorted(self.pools)})")
        self.pools[name].sched.add_agent(agent_id, slots)
        self._agent_pool[agent_id] = name
        return name

    def remove_agent(self, agent_id: str) -> None:
        name = self._agent_pool.pop(agent_id, None)
        if name is not None:
            self.pools[name].sched.remove_agent(agent_id)

    def set_agent_enabled(self, agent_id: str, enabled: bool) -> None:
        name = self._agent_pool.get(agent_id)
        if name is not None:
            self.pools[name].sched.set_agent_enabled(agent_id, enabled)

    def set_slot_enabled(self, agent_id: str, slot: int, enabled: bool) -> bool:
        name = self._agent_pool.get(agent_id)
        return name is not None and bool(self.pools[name].sched.set_slot_enabled(agent_id, int(slot), enabled))

    # ---------------------------------------------------------------- requests
    def add_request(self, alloc_id: str, job_id: str, slots: int, priority: int = 42, weight: float = 1.0,
                    order: int = 0, preemptible: bool = True, excluded_agents: Optional[List[str]] = None,
                    pool: Optional[str] = None) -> str:
        name = self.resolve(pool, slots)
        self.pools[name].sched.add_request(alloc_id, job_id, slots, priority, weight, order, preemptible,
                                           list(excluded_agents or []))
        self._req_pool[alloc_id] = name
        return name

    def remove_request(self, alloc_id: str) -> None:
        name = self._req_pool.pop(alloc_id, None)
        if name is not None:
            self.pools[name].sched.remove_request(alloc_id)

    def set_priority(self, job_id: str, priority: int) -> None:
        for p in self.pools.values():
            p.sched.set_priority(job_id, priority)

    def set_weight(self, job_id: str, weight: float) -> None:
        for p in self.pools.values():
            p.sched.set_weight(job_id, weight)

    def set_max_slots(self, job_id: str, max_slots: Optional[int]) -> None:
        """Fair-share group cap of a job (experiment ``resources.max_slots``; None: uncapped)."""
        for p in self.pools.values():
            p.sched.set_max_slots(job_id, -1 if max_slots is None else int(max_slots))

    def schedule(self) -> Dict[str, List[str]]:
        out: Dict[str, List[str]] = {"allocated": [], "preempt": []}
        for p in self.pools.values():
            d = p.sched.schedule()
            out["allocated"] += list(d["allocated"])
            out["preempt"] += list(d["preempt"])
        return out

    def requests(self, pool: Optional[str] = None) -> Dict[str, Dict[str, Any]]:
        out: Dict[str, Dict[str, Any]] = {}
        for name, p in self.pools.items():
            if pool is not None and name != pool:
                continue
            for aid, r in p.sched.requests().items():
                r = dict(r)
                r["resource_pool"] = name
                out[aid] = r
        return out

    def agents(self) -> Dict[str, Dict[str, Any]]:
        out: Dict[str, Dict[str, Any]] = {}
        for name, p in self.pools.items():
            for aid, a in p.sched.agents().items():
                a = dict(a)
                a["resource_pool"] = name
                out[aid] = a
        return out

    @property
    def total_slots(self) -> int:
        return sum(p.sched.total_slots for p in self.pools.values())

    @property
    def used_slots(self) -> int:
        return sum(p.sched.used_slots for p in self.pools.values())

    def summary(self) -> List[Dict[str, Any]]:
        rows = []
        for name, p in self.pools.items():
            ags = p.sched.agents()
            rows.append({"name": name, "description": p.description, "scheduler_type": p.policy,
                         "scheduler_fitting_policy": p.fit, "preemption": p.preemption,
                         "slots_available": p.sched.total_slots, "slots_used": p.sched.used_slots,
                         "num_agents": len(ags), "default_compute_pool": name == self.default_compute,
                         "default_aux_pool": name == self.default_aux})
        return rows
