"""Scheduler parity pinned to the reference's Go test vectors.

Fair share: every case of master/internal/rm/agentrm/fair_share_test.go replayed through
``_native.fairshare_decide`` (the decision function the live pool uses).  The Go mocks: a task's
group is its ``Group`` or, without one, a group of its own with weight 0 (Go zero value, as are
unset MaxSlots / Weight of listed groups); an ``AllocatedAgent`` task is already scheduled but holds
no device (ContainerStarted unset), so every agent shows all its slots free.

Priority: cases of priority_test.go replayed through the stateful ``Scheduler`` (allocations applied
between passes like the Go tests' AllocateTasks / RemoveTask helpers)."""

import pytest

from determined_amd._native import load as _load_native

_native = _load_native()
INF = -1


def _fs(tasks, groups, agents):
    """tasks: (id, group or None, slots, allocated, non_preemptible, blocked)."""
    rows = []
    for t in tasks:
        tid, group, slots = t[0], t[1], t[2]
        allocated = len(t) > 3 and t[3]
        nonpre = len(t) > 4 and t[4]
        blocked = list(t[5]) if len(t) > 5 else []
        rows.append((tid, group or tid, slots, bool(allocated), not nonpre, blocked))
    g = {name: (float(w), int(m)) for name, (w, m) in groups.items()}
    alloc, release = _native.fairshare_decide(rows, g, agents)
    return sorted(alloc), sorted(release)


# name: (agents, groups {id: (weight, max_slots)}, tasks, expected allocate, expected release)
FAIR_SHARE = {
    "MaxSlots": ({"agent": 4}, {"group1": (1, 1), "group2": (0, INF)},
                 [("task1", "group1", 1), ("task2", "group1", 1), ("task3", "group1", 1), ("task4", "group1", 1),
                  ("task5", "group2", 1), ("task6", "group2", 1), ("task7", "group2", 1), ("task8", "group2", 1)],
                 ["task1", "task5", "task6", "task7"], []),
    "Weights": ({"agent": 8}, {"group1": (10, 100), "group2": (30, 100)},
                [("task1", "group1", 1), ("task2", "group1", 1), ("task3", "group1", 1)] +
                [(f"task{i}", "group2", 1) for i in range(4, 11)],
                ["task1", "task2", "task4", "task5", "task6", "task7", "task8", "task9"], []),
    "MultiSlot": ({"agent1": 4, "agent2": 4}, {"group1": (0, INF), "group2": (0, INF)},
                  [("task1", "group1", 4), ("task2", "group2", 4)], ["task1", "task2"], []),
    "MaxSlotsReleaseAllocatedTasks": ({"agent": 4}, {"group1": (1, 2)},
                                      [(f"task{i}", "group1", 1, True) for i in range(1, 5)], [], ["task1", "task2"]),
    "Unscheduled": ({"agent1": 2, "agent2": 2}, {"group1": (1, 2)},
                    [("task1", "group1", 2), ("task2", "group1", 1, True), ("task3", "group1", 1, True)], [], []),
    "MultiSlotDeadlock": ({"agent": 2}, {"group1": (0, INF), "group2": (0, INF)},
                          [("task1", "group1", 2), ("task2", "group2", 2)], ["task1"], []),
    "BigTask": ({"agent": 4}, {"group1": (0, INF), "group2": (0, INF)},
                [("task1", "group1", 5), ("task2", "group2", 4)], ["task2"], []),
    "ActiveTasks": ({"agent1": 4, "agent2": 3}, {f"group{i}": (0, INF) for i in range(1, 5)},
                    [("task1", "group1", 3), ("task2", "group2", 1), ("task3", "group2", 1, True),
                     ("task4", "group3", 4), ("task5", "group4", 1)], ["task1", "task2", "task5"], []),
    "Nilgroup": ({"agent": 4}, {}, [("task1", None, 4, True), ("task2", None, 1, True)], [], ["task1"]),
    "Preemptible": ({"agent": 1}, {}, [("task1", None, 1, True), ("task2", None, 1, True)], [], ["task2"]),
    "HonorsNonPreemptibleInAGroup": ({"agent": 1}, {"group1": (1, 2)},
                                     [("task1", "group1", 1, True), ("task2", "group1", 1, True, True)], [], ["task1"]),
    "HonorsNonPreemptibleInAGroupReversed": ({"agent": 1}, {"group1": (1, 2)},
                                             [("task1", "group1", 1, True, True), ("task2", "group1", 1, True)], [],
                                             ["task2"]),
    "HonorsNonPreemptibleNilGroup": ({"agent": 1}, {},
                                     [("task1", None, 1, True), ("task2", None, 1, True, True)], [], ["task1"]),
    "HonorsNonPreemptibleNilGroupReversed": ({"agent": 1}, {},
                                             [("task1", None, 1, True, True), ("task2", None, 1, True)], [], ["task2"]),
    "Blocklist": ({"agent": 1}, {"group0": (0, INF), "group1": (0, INF)},
                  [("task0.1", "group0", 1, False, False, ["agent"]), ("task1.1", "group1", 1)], ["task1.1"], []),
    "BlocklistMultiple": ({f"agent{i}": 4 for i in range(4)}, {"group0": (0, INF), "group1": (0, INF)},
                          [("task0.1", "group0", 8, False, False, ["agent2", "agent3"]),
                           ("task1.1", "group1", 8, False, False, ["agent2", "agent3"])], ["task0.1", "task1.1"], []),
    "BlocklistPreemptible": ({"agent0": 1, "agent1": 1}, {},
                             [("task0.1", None, 1, False, False, ["agent0", "agent1"]), ("task1.1", None, 1, True),
                              ("task2.1", None, 1, False, False, ["agent0"]), ("task3.1", None, 1, True)],
                             ["task2.1"], ["task3.1"]),
    "BlocklistDontPreempt": ({"agent0": 1}, {},
                             [("task0.1", None, 1, False, False, ["agent0"]), ("task1.1", None, 1, False, False, ["agent0"]),
                              ("task2.1", None, 1, False, False, ["agent0"]), ("task3.1", None, 1, True)], [], []),
    "BlocklistEqual": ({"agent0": 1}, {},
                       [("task0.1", None, 1, False, False, ["agent0"]), ("task1.1", None, 1, True),
                        ("task2.1", None, 1, True), ("task3.1", None, 1, True)], [], ["task2.1", "task3.1"]),
}


@pytest.mark.parametrize("name", sorted(FAIR_SHARE))
def test_fair_share_go_vectors(name):
    agents, groups, tasks, want_alloc, want_release = FAIR_SHARE[name]
    alloc, release = _fs(tasks, groups, agents)
    assert alloc == sorted(want_alloc), (name, alloc)
    assert release == sorted(want_release), (name, release)


def test_live_pool_places_fair_share_decisions_without_overcommit():
    """BlocklistMultiple in the live pool: the decision starts both 8-slot tasks, the pool places the
    first and keeps the second queued (the reference's allocateResources refuses it the same way)."""
    s = _native.Scheduler(_native.Policy.FAIR_SHARE)
    for i in range(4):
        s.add_agent(f"agent{i}", 4)
    s.add_request("task0.1", "group0", 8, order=0, excluded_agents=["agent2", "agent3"])
    s.add_request("task1.1", "group1", 8, order=1, excluded_agents=["agent2", "agent3"])
    d = s.schedule()
    assert d["allocated"] == ["task0.1"] and d["preempt"] == []
    s.remove_request("task0.1")
    assert s.schedule()["allocated"] == ["task1.1"]


def test_live_pool_max_slots_caps_a_job():
    s = _native.Scheduler(_native.Policy.FAIR_SHARE)
    s.add_agent("a", 8)
    for i in range(6):
        s.add_request(f"e1.{i}", "exp1", 1, order=i)
    s.set_max_slots("exp1", 2)
    assert sorted(s.schedule()["allocated"]) == ["e1.0", "e1.1"]


# ------------------------------------------------------------------------------------------ priority
def _prio_sched(agents, preemption):
    s = _native.Scheduler(_native.Policy.PRIORITY, preemption=preemption)
    for a, n in agents.items():
        s.add_agent(a, n)
    return s


def test_priority_preemption_disabled_backfills_lower_priority():
    """TestPrioritySchedulingPreemptionDisabled: higher-priority 1 + 0 + 4 slots and lower 1 + 0 start,
    the lower 4-slot task does not fit."""
    s = _prio_sched({"agent1": 4, "agent2": 4}, False)
    tasks = [("task1", 50, 4), ("task2", 50, 1), ("task3", 40, 1), ("task4", 40, 0), ("task5", 40, 4), ("task6", 50, 0)]
    for i, (tid, prio, slots) in enumerate(tasks):
        s.add_request(tid, f"g{prio}", slots, priority=prio, order=i)
    assert sorted(s.schedule()["allocated"]) == ["task2", "task3", "task4", "task5", "task6"]


def test_priority_higher_priority_blocks_lower_when_it_cannot_fit():
    """TestPrioritySchedulingPreemptionDisabledHigherPriorityBlocksLowerPriority: a 12-slot higher-priority
    task that can never fit on 2x4 slots blocks the lower-priority ones."""
    s = _prio_sched({"agent1": 4, "agent2": 4}, False)
    for i, (tid, prio, slots) in enumerate([("task1", 50, 4), ("task2", 50, 1), ("task3", 40, 12)]):
        s.add_request(tid, f"g{prio}", slots, priority=prio, order=i)
    assert s.schedule()["allocated"] == []


def test_priority_lower_priority_must_wait():
    """TestPrioritySchedulingPreemptionDisabledLowerPriorityMustWait: 3 of the 4 higher-priority slots
    start; nothing more while they run; once they end the 2-slot higher and the lower task start."""
    s = _prio_sched({"agent1": 4}, False)
    tasks = [("task1", 50, 1), ("task2", 40, 1), ("task3", 40, 1), ("task4", 40, 1), ("task5", 40, 2)]
    for i, (tid, prio, slots) in enumerate(tasks):
        s.add_request(tid, f"g{prio}", slots, priority=prio, order=i)
    first = s.schedule()["allocated"]
    assert sorted(first) == ["task2", "task3", "task4"]
    assert s.schedule()["allocated"] == []
    for t in first:
        s.remove_request(t)
    assert sorted(s.schedule()["allocated"]) == ["task1", "task5"]


def test_priority_add_tasks_after_allocation():
    """TestPrioritySchedulingPreemptionDisabledAddTasks: after the first pass, three new 1-slot
    lower-priority tasks: two fit in the remaining slots."""
    s = _prio_sched({"agent1": 4, "agent2": 4}, False)
    tasks = [("task1", 50, 4), ("task2", 50, 1), ("task3", 40, 1), ("task4", 40, 0), ("task5", 40, 4), ("task6", 50, 0)]
    for i, (tid, prio, slots) in enumerate(tasks):
        s.add_request(tid, f"g{prio}", slots, priority=prio, order=i)
    s.schedule()
    for i, tid in enumerate(["task7", "task8", "task9"]):
        s.add_request(tid, "g50", 1, priority=50, order=10 + i)
    assert sorted(s.schedule()["allocated"]) == ["task7", "task8"]


def test_priority_preemption_evicts_lower_priority():
    """With preemption enabled, a higher-priority task that does not fit evicts lower-priority
    preemptible tasks (newest first) and starts once they release."""
    s = _prio_sched({"agent1": 4}, True)
    for i in range(4):
        s.add_request(f"low{i}", "glow", 1, priority=50, order=i)
    assert len(s.schedule()["allocated"]) == 4
    s.add_request("high", "ghigh", 2, priority=40, order=10)
    d = s.schedule()
    assert d["allocated"] == [] and sorted(d["preempt"]) == ["low2", "low3"]
    for v in d["preempt"]:
        s.remove_request(v)
    assert s.schedule()["allocated"] == ["high"]
