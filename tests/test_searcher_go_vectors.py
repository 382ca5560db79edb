"""Search methods pinned to the reference Go tests' exact expectations
(``master/pkg/searcher/{adaptive_asha,asha,asha_stopping}_test.go``): bracket sizing vectors, and
value simulations where every trial's sequence of validation lengths is fixed by its metric.

The driver mirrors ``util_test.go checkValueSimulation``: one FIFO queue of searcher operations;
Create takes the next predefined trial; ValidateAfter checks the requested length against the
trial's script and answers with its metric (or an early exit on the scripted op); Close checks the
trial ran its whole script; the engine is snapshotted and restored after every validation (as
``saveAndReload``).  ``checkSimulation`` (ConstantValidation) compares the multiset of per-trial
length sequences.
"""

import pytest

from determined_amd.searcher import Searcher

EXIT = True

# (Go test, case name, searcher config (Go defaults applied by Searcher / expconf), [(lengths, metric[, EXIT])])
VALUE_CASES = [
    ("TestASHASearchMethod", "smaller is better", {'name': 'async_halving', 'smaller_is_better': True, 'num_rungs': 3, 'max_length': 9000, 'max_trials': 12, 'divisor': 3.0},
     [("1000 3000 9000", 0.01), ("1000 3000", 0.02), ("1000 3000", 0.03), ("1000 3000", 0.04), ("1000", 0.05), ("1000", 0.06), ("1000", 0.07), ("1000", 0.08), ("1000", 0.09), ("1000", 0.1), ("1000", 0.11), ("1000", 0.12)]),
    ("TestASHASearchMethod", "early exit -- smaller is better", {'name': 'async_halving', 'smaller_is_better': True, 'num_rungs': 3, 'max_length': 9000, 'max_trials': 12, 'divisor': 3.0},
     [("1000 3000 9000", 0.01), ("1000 3000", 0.02), ("1000 3000", 0.03, EXIT), ("1000 3000", 0.04), ("1000", 0.05), ("1000", 0.06), ("1000", 0.07), ("1000", 0.08), ("1000", 0.09), ("1000", 0.1), ("1000", 0.11), ("1000", 0.12)]),
    ("TestASHASearchMethod", "smaller is not better", {'name': 'async_halving', 'smaller_is_better': False, 'num_rungs': 3, 'max_length': 9000, 'max_trials': 12, 'divisor': 3.0},
     [("1000 3000 9000", 0.12), ("1000 3000", 0.11), ("1000 3000", 0.1), ("1000 3000", 0.09), ("1000", 0.08), ("1000", 0.07), ("1000", 0.06), ("1000", 0.05), ("1000", 0.04), ("1000", 0.03), ("1000", 0.02), ("1000", 0.01)]),
    ("TestASHASearchMethod", "early exit -- smaller is not better", {'name': 'async_halving', 'smaller_is_better': False, 'num_rungs': 3, 'max_length': 9000, 'max_trials': 12, 'divisor': 3.0},
     [("1000 3000 9000", 0.12), ("1000 3000", 0.11), ("1000 3000", 0.1, EXIT), ("1000 3000", 0.09), ("1000", 0.08), ("1000", 0.07), ("1000", 0.06), ("1000", 0.05), ("1000", 0.04), ("1000", 0.03), ("1000", 0.02), ("1000", 0.01)]),
    ("TestASHASearchMethod", "async promotions", {'name': 'async_halving', 'smaller_is_better': True, 'num_rungs': 3, 'max_length': 9000, 'max_trials': 12, 'divisor': 3.0},
     [("1000 3000", 0.1), ("1000", 0.11), ("1000", 0.12, EXIT), ("1000 3000 9000", 0.01), ("1000 3000", 0.02), ("1000 3000", 0.03), ("1000 3000", 0.04), ("1000", 0.05), ("1000", 0.06), ("1000", 0.07), ("1000", 0.08), ("1000", 0.09)]),
    ("TestASHASearchMethod", "single rung bracket", {'name': 'async_halving', 'smaller_is_better': True, 'num_rungs': 1, 'max_length': 9000, 'max_trials': 4, 'divisor': 3.0},
     [("9000", 0.05), ("9000", 0.06), ("9000", 0.07), ("9000", 0.08)]),
    ("TestAdaptiveASHASearchMethod", "smaller is better", {'name': 'adaptive_asha', 'smaller_is_better': True, 'max_length': 900, 'max_trials': 5, 'mode': 'standard', 'max_rungs': 2, 'divisor': 3.0},
     [("300 900", 0.1), ("300", 0.2), ("300", 0.3), ("900", 0.4), ("900", 0.5)]),
    ("TestAdaptiveASHASearchMethod", "early exit -- smaller is better", {'name': 'adaptive_asha', 'smaller_is_better': True, 'max_length': 900, 'max_trials': 5, 'mode': 'standard', 'max_rungs': 2, 'divisor': 3.0},
     [("300 900", 0.1), ("300", 0.2, EXIT), ("300", 0.3), ("900", 0.4), ("900", 0.5)]),
    ("TestAdaptiveASHASearchMethod", "smaller is not better", {'name': 'adaptive_asha', 'smaller_is_better': False, 'max_length': 900, 'max_trials': 5, 'mode': 'standard', 'max_rungs': 2, 'divisor': 3.0},
     [("300 900", 0.5), ("300", 0.4), ("300", 0.3), ("900", 0.2), ("900", 0.1)]),
    ("TestAdaptiveASHASearchMethod", "early exit -- smaller is not better", {'name': 'adaptive_asha', 'smaller_is_better': False, 'max_length': 900, 'max_trials': 5, 'mode': 'standard', 'max_rungs': 2, 'divisor': 3.0},
     [("300 900", 0.5), ("300", 0.4, EXIT), ("300", 0.3), ("900", 0.2), ("900", 0.1)]),
    ("TestAdaptiveASHAStoppingSearchMethod", "smaller is better", {'name': 'adaptive_asha', 'smaller_is_better': True, 'max_length': 900, 'max_trials': 5, 'mode': 'standard', 'max_rungs': 2, 'divisor': 3.0, 'stop_once': True},
     [("300 900", 0.1), ("300", 0.2), ("300", 0.3), ("900", 0.4), ("900", 0.5)]),
    ("TestAdaptiveASHAStoppingSearchMethod", "early exit -- smaller is better", {'name': 'adaptive_asha', 'smaller_is_better': True, 'max_length': 900, 'max_trials': 5, 'mode': 'standard', 'max_rungs': 2, 'divisor': 3.0, 'stop_once': True},
     [("300 900", 0.1), ("300", 0.2, EXIT), ("300", 0.3), ("900", 0.4), ("900", 0.5)]),
    ("TestAdaptiveASHAStoppingSearchMethod", "smaller is not better", {'name': 'adaptive_asha', 'smaller_is_better': False, 'max_length': 900, 'max_trials': 5, 'mode': 'standard', 'max_rungs': 2, 'divisor': 3.0, 'stop_once': True},
     [("300 900", 0.1), ("300 900", 0.2), ("300 900", 0.3), ("900", 0.4), ("900", 0.5)]),
    ("TestAdaptiveASHAStoppingSearchMethod", "early exit -- smaller is not better", {'name': 'adaptive_asha', 'smaller_is_better': False, 'max_length': 900, 'max_trials': 5, 'mode': 'standard', 'max_rungs': 2, 'divisor': 3.0, 'stop_once': True},
     [("300 900", 0.1), ("300", 0.2, EXIT), ("300 900", 0.3), ("900", 0.4), ("900", 0.5)]),
    ("TestASHAStoppingSearchMethod", "smaller is better", {'name': 'async_halving', 'smaller_is_better': True, 'num_rungs': 3, 'max_length': 9000, 'max_trials': 12, 'divisor': 3.0, 'stop_once': True},
     [("1000 3000 9000", 0.01), ("1000", 0.02), ("1000", 0.03), ("1000", 0.04), ("1000", 0.05), ("1000", 0.06), ("1000", 0.07), ("1000", 0.08), ("1000", 0.09), ("1000", 0.1), ("1000", 0.11), ("1000", 0.12)]),
    ("TestASHAStoppingSearchMethod", "smaller is better (round robin)", {'name': 'async_halving', 'smaller_is_better': True, 'num_rungs': 3, 'max_length': 9000, 'max_trials': 12, 'divisor': 3.0, 'stop_once': True},
     [("1000 3000 9000", 0.01), ("1000", 0.02), ("1000", 0.03), ("1000", 0.04), ("1000 3000 9000", 0.01), ("1000", 0.02), ("1000", 0.03), ("1000", 0.04), ("1000 3000 9000", 0.01), ("1000", 0.02), ("1000", 0.03), ("1000", 0.04)]),
    ("TestASHAStoppingSearchMethod", "smaller is not better", {'name': 'async_halving', 'smaller_is_better': False, 'num_rungs': 3, 'max_length': 9000, 'max_trials': 12, 'divisor': 3.0, 'stop_once': True},
     [("1000 3000 9000", 0.01), ("1000 3000 9000", 0.02), ("1000 3000 9000", 0.03), ("1000 3000 9000", 0.04), ("1000 3000 9000", 0.05), ("1000 3000 9000", 0.06), ("1000 3000 9000", 0.07), ("1000 3000 9000", 0.08), ("1000 3000 9000", 0.09), ("1000 3000 9000", 0.1), ("1000 3000 9000", 0.11), ("1000 3000 9000", 0.12)]),
    ("TestASHAStoppingSearchMethod", "smaller is not better (round robin)", {'name': 'async_halving', 'smaller_is_better': False, 'num_rungs': 3, 'max_length': 9000, 'max_trials': 12, 'divisor': 3.0, 'stop_once': True},
     [("1000 3000 9000", 0.01), ("1000 3000 9000", 0.02), ("1000 3000 9000", 0.03), ("1000 3000 9000", 0.04), ("1000", 0.01), ("1000", 0.02), ("1000 3000", 0.03), ("1000 3000 9000", 0.04), ("1000", 0.01), ("1000", 0.02), ("1000 3000", 0.03), ("1000 3000 9000", 0.04)]),
    ("TestASHAStoppingSearchMethod", "early exit -- smaller is better (round robin)", {'name': 'async_halving', 'smaller_is_better': True, 'num_rungs': 3, 'max_length': 9000, 'max_trials': 12, 'divisor': 3.0, 'stop_once': True},
     [("1000 3000 9000", 0.01), ("1000", 0.02), ("1000", 0.03), ("1000", 0.04), ("1000 3000", 0.01, EXIT), ("1000", 0.02), ("1000", 0.03), ("1000", 0.04), ("1000 3000 9000", 0.01), ("1000", 0.02), ("1000", 0.03), ("1000", 0.04)]),
    ("TestASHAStoppingSearchMethod", "early exit -- smaller is not better (round robin)", {'name': 'async_halving', 'smaller_is_better': False, 'num_rungs': 3, 'max_length': 9000, 'max_trials': 12, 'divisor': 3.0, 'stop_once': True},
     [("1000 3000 9000", 0.01), ("1000 3000 9000", 0.02), ("1000 3000 9000", 0.03), ("1000 3000", 0.04, EXIT), ("1000", 0.01), ("1000", 0.02), ("1000 3000 9000", 0.03), ("1000 3000 9000", 0.04), ("1000", 0.01), ("1000", 0.02), ("1000 3000 9000", 0.03), ("1000 3000 9000", 0.04)]),
    ("TestASHAStoppingSearchMethod", "single rung bracket", {'name': 'async_halving', 'smaller_is_better': True, 'num_rungs': 1, 'max_length': 9000, 'max_trials': 4, 'divisor': 3.0, 'stop_once': True},
     [("9000", 0.05), ("9000", 0.06), ("9000", 0.07), ("9000", 0.08)]),
]

EXPCONF_DEFAULTS = {
    "async_halving": {"max_concurrent_trials": 16, "stop_once": False, "divisor": 4.0},
    "adaptive_asha": {"max_concurrent_trials": 16, "stop_once": False, "divisor": 4.0, "mode": "standard",
                      "max_rungs": 5},
}


def _config(cfg):
    out = {"metric": "metric", "smaller_is_better": True, **EXPCONF_DEFAULTS[cfg["name"]], **cfg}
    return out


def check_value_simulation(cfg, expected):
    s = Searcher(_config(cfg), {}, seed=0)
    script = [([int(x) for x in lengths.split()], metric, bool(rest and rest[0]))
              for lengths, metric, *rest in expected]
    pending = list(s.initial_operations())
    trial_of, op_idx, exited = {}, {}, set()
    nxt = 0
    while pending:
        op = pending.pop(0)
        rid = op["request_id"]
        if op["type"] == "create":
            assert nxt < len(script), "search method created too many trials"
            trial_of[rid], op_idx[rid] = nxt, 0
            nxt += 1
            ops = s.trial_created(rid)
        elif op["type"] == "validate_after":
            if rid in exited:
                continue
            lengths, metric, early = script[trial_of[rid]]
            i = op_idx[rid]
            assert i < len(lengths), f"trial {trial_of[rid] + 1}: ran out of expected ops (asked {op['length']})"
            assert op["length"] == lengths[i], f"trial {trial_of[rid] + 1}: wanted {lengths[i]} got {op['length']}"
            if early and i == len(lengths) - 1:
                exited.add(rid)
                ops = s.trial_exited_early(rid, "USER_REQUESTED_STOP")
            else:
                ops = s.validation_completed(rid, metric, op["length"])
            op_idx[rid] += 1
            snap = s.snapshot()  # saveAndReload
            s2 = Searcher(_config(cfg), {}, seed=0)
            s2.restore(snap)
            s = s2
        elif op["type"] == "close":
            lengths = script[trial_of[rid]][0]
            assert op_idx[rid] == len(lengths), f"trial {trial_of[rid] + 1} closed with ops {lengths[op_idx[rid]:]} left"
            ops = s.trial_closed(rid)
        elif op["type"] == "shutdown":
            ops = []
        else:
            raise AssertionError(f"unexpected operation {op}")
        pending += ops
    assert nxt == len(script), f"created {nxt} trials, expected {len(script)}"
    for rid, t in trial_of.items():
        assert op_idx[rid] == len(script[t][0]), f"incomplete trial {t + 1}"


@pytest.mark.parametrize("test,name,cfg,expected", VALUE_CASES, ids=[f"{c[0]}::{c[1]}" for c in VALUE_CASES])
def test_value_simulation_matches_go(test, name, cfg, expected):
    check_value_simulation(cfg, expected)


def test_bracket_max_trials_vectors():
    from determined_amd._native import load

    n = load()
    assert n.bracket_max_trials(20, 3.0, [3, 2, 1]) == [12, 5, 3]
    assert n.bracket_max_trials(50, 3.0, [4, 3]) == [35, 15]
    assert n.bracket_max_trials(50, 4.0, [3, 2]) == [37, 13]
    assert n.bracket_max_trials(100, 4.0, [4, 3, 2]) == [70, 22, 8]


def test_bracket_max_concurrent_trials_vectors():
    from determined_amd._native import load

    n = load()
    assert n.bracket_max_concurrent(0, 3.0, [9, 3, 1]) == [3, 3, 3]
    assert n.bracket_max_concurrent(11, 3.0, [9, 3, 1]) == [4, 4, 3]
    assert n.bracket_max_concurrent(0, 4.0, [40, 10]) == [10, 10]


def _constant_simulation(cfg, trial_id_metric=False):
    """checkSimulation, FIFO order: ConstantValidation (every validation reports 1.0) or TrialIDMetric
    (a trial reports its creation index, so later trials are worse)."""
    s = Searcher(_config(cfg), {}, seed=0)
    pending = list(s.initial_operations())
    runs, ids = {}, {}
    while pending:
        op = pending.pop(0)
        rid = op["request_id"]
        if op["type"] == "create":
            runs[rid] = []
            ids[rid] = len(ids) + 1
            pending += s.trial_created(rid)
        elif op["type"] == "validate_after":
            runs[rid].append(op["length"])
            pending += s.validation_completed(rid, float(ids[rid]) if trial_id_metric else 1.0, op["length"])
        elif op["type"] == "close":
            pending += s.trial_closed(rid)
    return sorted(tuple(v) for v in runs.values())


# asha_test.go TestASHASearcher{Records,Batches,Epochs} and asha_stopping_test.go equivalents: the
# multiset of per-trial length sequences (units are the config's own: 576000 records, 9000 batches, 12 epochs)
@pytest.mark.parametrize("max_length,rungs", [(576000, (64000, 192000, 576000)), (9000, (1000, 3000, 9000)),
                                              (12, (1, 4, 12))])
def test_asha_constant_simulation(max_length, rungs):
    got = _constant_simulation({"name": "async_halving", "num_rungs": 3, "max_length": max_length, "divisor": 3.0,
                                "max_trials": 12})
    a, b, c = rungs
    want = sorted([(a,)] * 8 + [(a, b)] * 3 + [(a, b, c)])
    assert got == want


@pytest.mark.parametrize("max_length,rungs", [(576000, (64000, 192000, 576000)), (9000, (1000, 3000, 9000)),
                                              (12, (1, 4, 12))])
def test_asha_stopping_constant_simulation(max_length, rungs):
    got = _constant_simulation({"name": "async_halving", "num_rungs": 3, "max_length": max_length, "divisor": 3.0,
                                "max_trials": 12, "stop_once": True, "max_concurrent_trials": 2},
                               trial_id_metric=True)
    a, b, c = rungs
    assert got == sorted([(a,)] * 11 + [(a, b, c)])
