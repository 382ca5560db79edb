"""Native search methods (C++): behaviour checks modelled on master/pkg/searcher/*_test.go."""

import math

import pytest

from determined_amd.searcher import Searcher, decode_sample, flatten_hparams, simulate

HP = {
    "lr": {"type": "log", "minval": -4, "maxval": -1, "base": 10},
    "layers": {"type": "int", "minval": 1, "maxval": 8},
    "opt": {"type": "categorical", "vals": ["sgd", "adam", {"name": "lamb"}]},
    "nested": {"dropout": {"type": "double", "minval": 0.0, "maxval": 0.5}, "const": {"type": "const", "val": [1, 2]}},
    "gbs": 32,
}


def metric(hp, length):
    # better with more training and smaller lr exponent distance from 1e-2
    return abs(math.log10(hp["lr"]) + 2) + 1.0 / (1 + length) + hp["layers"] * 0.01


def test_hparam_sampling_types_and_ranges():
    s = Searcher({"name": "random", "max_length": 10, "max_trials": 50, "max_concurrent_trials": 50,
                  "metric": "m"}, HP, seed=3)
    ops = [o for o in s.initial_operations() if o["type"] == "create"]
    assert len(ops) == 50
    for o in ops:
        hp = o["hparams"]
        assert 1e-4 <= hp["lr"] <= 1e-1
        assert isinstance(hp["layers"], int) and 1 <= hp["layers"] <= 8
        assert hp["opt"] in ("sgd", "adam", {"name": "lamb"})
        assert 0 <= hp["nested"]["dropout"] <= 0.5 and hp["nested"]["const"] == [1, 2]
        assert hp["gbs"] == 32
    assert len({o["hparams"]["lr"] for o in ops}) == 50


def test_random_search_respects_max_concurrency_and_trials():
    r = simulate({"name": "random", "max_length": 5, "max_trials": 7, "max_concurrent_trials": 3, "metric": "m"},
                 HP, metric)
    assert len(r["trials"]) == 7
    assert all(t["lengths"] == [5] and t["closed"] for t in r["trials"].values())
    assert r["progress"] == pytest.approx(1.0)


def test_single_search():
    r = simulate({"name": "single", "max_length": 9, "metric": "m"}, HP, metric)
    assert len(r["trials"]) == 1 and next(iter(r["trials"].values()))["lengths"] == [9]


def test_grid_search_cartesian_product():
    hp = {"a": {"type": "int", "minval": 0, "maxval": 10, "count": 3},
          "b": {"type": "categorical", "vals": [1, 2]},
          "c": {"type": "log", "minval": -2, "maxval": 0, "base": 10, "count": 2},
          "d": 5}
    r = simulate({"name": "grid", "max_length": 4, "max_concurrent_trials": 2, "metric": "m"}, hp,
                 lambda h, l: 0.0)
    combos = sorted((t["hparams"]["a"], t["hparams"]["b"], round(t["hparams"]["c"], 6)) for t in r["trials"].values())
    assert combos == sorted((a, b, c) for a in (0, 5, 10) for b in (1, 2) for c in (0.01, 1.0))


def test_asha_promotes_top_fraction():
    cfg = {"name": "async_halving", "num_rungs": 3, "max_length": 16, "max_trials": 16, "divisor": 4,
           "max_concurrent_trials": 16, "metric": "m", "smaller_is_better": True}
    r = simulate(cfg, HP, metric)
    trials = list(r["trials"].values())
    assert len(trials) == 16
    rung_lengths = sorted({l for t in trials for l in t["lengths"]})
    assert rung_lengths == [1, 4, 16]
    reached_top = [t for t in trials if 16 in t["lengths"]]
    reached_mid = [t for t in trials if 4 in t["lengths"]]
    assert 1 <= len(reached_top) <= len(reached_mid) <= 8
    assert all(t["closed"] for t in trials)
    # promoted trials are the best at their rung
    scores = sorted((metric(t["hparams"], 1), id(t)) for t in trials)
    best_mid = {id(t) for t in reached_mid}
    assert scores[0][1] in best_mid


def test_asha_stop_once():
    cfg = {"name": "async_halving", "num_rungs": 3, "max_length": 16, "max_trials": 16, "divisor": 4,
           "max_concurrent_trials": 4, "stop_once": True, "metric": "m"}
    r = simulate(cfg, HP, metric)
    assert len(r["trials"]) == 16 and all(t["closed"] for t in r["trials"].values())


@pytest.mark.parametrize("mode,expect_brackets", [("aggressive", 1), ("standard", 2), ("conservative", 3)])
def test_adaptive_asha_brackets(mode, expect_brackets):
    cfg = {"name": "adaptive_asha", "max_length": 64, "max_trials": 32, "max_concurrent_trials": 8,
           "mode": mode, "divisor": 4, "max_rungs": 5, "metric": "m"}
    s = Searcher(cfg, HP, seed=0)
    s.initial_operations()
    snap = s.snapshot()["engine"]["method"]
    assert len(snap["sub_search_states"]) == expect_brackets
    r = simulate(cfg, HP, metric)
    assert len(r["trials"]) == 32
    assert all(t["closed"] for t in r["trials"].values())


def test_adaptive_asha_cifar_config_32_trials_8_concurrent():
    # BASELINE config: CIFAR-10 adaptive_asha, 32 trials, max_concurrent_trials=8
    cfg = {"name": "adaptive_asha", "max_length": {"epochs": 32}, "max_trials": 32, "max_concurrent_trials": 8,
           "metric": "validation_error"}
    s = Searcher(cfg, HP, seed=1)
    creates = [o for o in s.initial_operations() if o["type"] == "create"]
    assert len(creates) == 8


def test_snapshot_restore_continues_identically():
    cfg = {"name": "adaptive_asha", "max_length": 32, "max_trials": 12, "max_concurrent_trials": 4, "metric": "m"}
    a = Searcher(cfg, HP, seed=5)
    ops = a.initial_operations()
    creates = [o for o in ops if o["type"] == "create"]
    for c in creates:
        a.trial_created(c["request_id"])
    snap = a.snapshot()
    b = Searcher(cfg, HP, seed=999)
    b.restore(snap)
    first = creates[0]["request_id"]
    length = [o["length"] for o in ops if o["type"] == "validate_after" and o["request_id"] == first][0]
    oa = a.validation_completed(first, 0.5, length)
    ob = b.validation_completed(first, 0.5, length)
    assert oa == ob


def test_invalid_hp_replaced_in_asha():
    cfg = {"name": "async_halving", "num_rungs": 2, "max_length": 4, "max_trials": 4, "max_concurrent_trials": 2,
           "metric": "m"}
    s = Searcher(cfg, {"x": {"type": "double", "minval": 0, "maxval": 1}}, seed=0)
    ops = s.initial_operations()
    rid = ops[0]["request_id"]
    s.trial_created(rid)
    new = s.trial_exited_early(rid, "invalid_hp")
    assert [o["type"] for o in new] == ["close", "create", "validate_after"]


def test_flatten_and_decode_roundtrip():
    flat, tables = flatten_hparams(HP)
    paths = [f["path"] for f in flat]
    assert "nested.dropout" in paths and "nested.const" in paths
    hp = decode_sample([("nested.dropout", 1, 0, 0.25), ("opt", 2, 2, 0.0), ("gbs", 2, 0, 0.0)], tables)
    assert hp == {"nested": {"dropout": 0.25}, "opt": {"name": "lamb"}, "gbs": 32}
