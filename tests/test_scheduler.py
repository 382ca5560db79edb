"""Native scheduler (C++): priority/preemption/backfill, fair share, round robin, gang fitting
(behaviours from master/internal/rm/agentrm/*_test.go)."""

from determined_amd._native import load

N = load()


def sched(policy="priority", preemption=True):
    p = {"priority": N.Policy.PRIORITY, "fair_share": N.Policy.FAIR_SHARE, "round_robin": N.Policy.ROUND_ROBIN}[policy]
    return N.Scheduler(p, N.Fit.BEST, preemption)


def test_packs_eight_single_slot_trials_on_one_node():
    s = sched()
    s.add_agent("mi355x", 8)
    for i in range(10):
        s.add_request(f"t{i}", f"exp1", 1, order=i)
    d = s.schedule()
    assert sorted(d["allocated"]) == sorted(f"t{i}" for i in range(8))
    used = sorted(sl for r in s.requests().values() if r["allocated"] for _, sls in r["assignment"] for sl in sls)
    assert used == list(range(8))
    s.remove_request("t0")
    assert s.schedule()["allocated"] == ["t8"]


def test_gang_schedules_eight_slot_trial():
    s = sched()
    s.add_agent("mi355x", 8)
    s.add_request("small", "e1", 1, order=0)
    s.add_request("big", "e2", 8, order=1)
    d = s.schedule()
    assert d["allocated"] == ["small"]  # big does not fit while small runs
    s.remove_request("small")
    d = s.schedule()
    assert d["allocated"] == ["big"]
    assert s.requests()["big"]["assignment"] == [("mi355x", list(range(8)))]


def test_multi_agent_dedicated_fit():
    s = sched()
    s.add_agent("n0", 8)
    s.add_agent("n1", 8)
    s.add_request("job16", "e", 16)
    assert s.schedule()["allocated"] == ["job16"]
    assert sorted(a for a, _ in s.requests()["job16"]["assignment"]) == ["n0", "n1"]
    s2 = sched()
    s2.add_agent("n0", 8)
    s2.add_agent("n1", 8)
    s2.add_request("odd12", "e", 12)  # not a multiple of per-agent slots -> unschedulable
    assert s2.schedule()["allocated"] == []


def test_priority_preemption():
    s = sched()
    s.add_agent("n", 8)
    s.add_request("low", "e_low", 8, priority=50, order=0)
    assert s.schedule()["allocated"] == ["low"]
    s.add_request("high", "e_high", 4, priority=10, order=1)
    d = s.schedule()
    assert d["allocated"] == [] and d["preempt"] == ["low"]
    s.remove_request("low")  # the preempted task checkpoints and exits
    assert s.schedule()["allocated"] == ["high"]


def test_priority_without_preemption_waits():
    s = sched(preemption=False)
    s.add_agent("n", 4)
    s.add_request("low", "a", 4, priority=50)
    s.schedule()
    s.add_request("high", "b", 4, priority=1, order=1)
    d = s.schedule()
    assert d == {"allocated": [], "preempt": []}


def test_fair_share_splits_between_jobs():
    """Reference fair_share.go semantics: tasks that fit nowhere right now are left out of the share
    computation (calculateGroupStates), so a full node is not rebalanced until a slot frees; then
    the starved job enters the share, the job above its share releases tasks (oldest first, like
    the reference's allocatedReqs order) and the starved job takes the freed slots."""
    s = sched("fair_share")
    s.add_agent("n", 8)
    for i in range(8):
        s.add_request(f"a{i}", "A", 1, order=i)
    assert len(s.schedule()["allocated"]) == 8
    for i in range(8):
        s.add_request(f"b{i}", "B", 1, order=100 + i)
    assert s.schedule() == {"allocated": [], "preempt": []}
    s.remove_request("a7")  # one A task finishes: B now fits and enters the share
    d = s.schedule()
    assert d["allocated"] == ["b0"] and d["preempt"] == ["a0", "a1", "a2"]
    for aid in d["preempt"]:
        s.remove_request(aid)
    d = s.schedule()
    assert d["allocated"] == ["b1", "b2", "b3"] and d["preempt"] == []


def test_round_robin_fifo_blocks():
    s = sched("round_robin")
    s.add_agent("n", 8)
    s.add_request("x", "1", 6, order=0)
    s.add_request("y", "2", 4, order=1)
    s.add_request("z", "3", 1, order=2)
    assert s.schedule()["allocated"] == ["x"]  # y blocks z (FIFO)


def test_disabled_slots_are_never_offered():
    """``det slot disable`` (reference agentrm slot enable/disable): a disabled slot is skipped by
    shared fits, removes the agent from whole-agent gang fits and from the pool's capacity; a
    slot disabled under a running allocation stays with it until it ends."""
    s = sched()
    s.add_agent("n", 4)
    assert s.set_slot_enabled("n", 1, False) and not s.set_slot_enabled("n", 9, False)
    assert s.total_slots == 3 and s.agents()["n"]["disabled_slots"] == [1]
    s.add_request("a", "e", 3, order=0)
    assert s.schedule()["allocated"] == ["a"]
    assert s.requests()["a"]["assignment"] == [("n", [0, 2, 3])]
    s.add_request("b", "e2", 1, order=1)
    assert s.schedule()["allocated"] == []  # the only free slot is disabled
    s.set_slot_enabled("n", 1, True)
    assert s.schedule()["allocated"] == ["b"]
    s.set_slot_enabled("n", 1, False)  # disabled while "b" holds it
    assert s.used_slots == 4
    s.remove_request("b")
    assert s.used_slots == 3 and s.total_slots == 3
    # whole-agent (multi-agent) gang fits skip agents with a disabled slot
    g = sched()
    g.add_agent("n0", 2)
    g.add_agent("n1", 2)
    g.set_slot_enabled("n1", 0, False)
    g.add_request("gang", "e", 4)
    assert g.schedule()["allocated"] == []
    g.set_slot_enabled("n1", 0, True)
    assert g.schedule()["allocated"] == ["gang"]
