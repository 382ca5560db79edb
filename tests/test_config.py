"""Experiment config defaults/validation (semantics of reference schemas/expconf/v0)."""

import pytest

from determined_amd import config


def test_defaults_match_reference_schema():
    cfg = config.parse({"searcher": {"name": "single", "metric": "loss", "max_length": {"batches": 10}},
                        "hyperparameters": {"lr": 0.1}})
    assert cfg["max_restarts"] == 5
    assert cfg["scheduling_unit"] == 100
    assert cfg["checkpoint_policy"] == "best"
    assert cfg["resources"]["slots_per_trial"] == 1
    assert cfg["optimizations"]["aggregation_frequency"] == 1
    assert cfg["checkpoint_storage"]["save_trial_best"] == 1
    assert cfg["checkpoint_storage"]["save_trial_latest"] == 1
    assert cfg["checkpoint_storage"]["save_experiment_best"] == 0
    assert cfg["searcher"]["smaller_is_better"] is True
    assert cfg["hyperparameters"]["lr"] == {"type": "const", "val": 0.1}
    assert isinstance(cfg["reproducibility"]["experiment_seed"], int)


def test_adaptive_asha_defaults():
    cfg = config.parse({"searcher": {"name": "adaptive_asha", "metric": "m", "max_length": {"epochs": 4},
                                     "max_trials": 32}})
    s = cfg["searcher"]
    assert (s["divisor"], s["max_rungs"], s["mode"], s["max_concurrent_trials"]) == (4, 5, "standard", 16)
    assert config.searcher_unit(cfg) == config.Unit.EPOCHS


@pytest.mark.parametrize("bad,msg", [
    ({"searcher": {"name": "random", "metric": "m", "max_length": 5}}, "max_trials"),
    ({"searcher": {"name": "nope", "metric": "m"}}, "is one of"),
    ({"searcher": {"name": "single", "max_length": 5}}, "metric"),
    ({"searcher": {"name": "single", "metric": "m", "max_length": {"hours": 3}}}, "max_length"),
    ({"searcher": {"name": "grid", "metric": "m", "max_length": 5},
      "hyperparameters": {"x": {"type": "double", "minval": 0, "maxval": 1}}}, "count"),
    ({"searcher": {"name": "single", "metric": "m", "max_length": 5},
      "hyperparameters": {"x": {"type": "int", "minval": 3, "maxval": 1}}}, "minval"),
    ({"searcher": {"name": "single", "metric": "m", "max_length": 5},
      "checkpoint_storage": {"type": "s3"}}, "bucket"),
])
def test_validation_errors(bad, msg):
    with pytest.raises(config.InvalidConfig) as e:
        config.parse(bad)
    assert msg in str(e.value)


def test_length_conversion():
    assert config.Length.parse({"records": 1000}).to_batches(64) == 16
    assert config.Length.parse({"epochs": 2}).to_batches(10, records_per_epoch=100) == 20
    assert config.Length.parse(7).to_batches(3) == 7


def test_yaml_roundtrip(tmp_path):
    p = tmp_path / "c.yaml"
    p.write_text("searcher:\n  name: single\n  metric: loss\n  max_length:\n    batches: 3\n"
                 "hyperparameters:\n  opt:\n    lr: 0.1\n    mom:\n      type: double\n      minval: 0\n      maxval: 1\n")
    cfg = config.parse(str(p))
    assert cfg["hyperparameters"]["opt"]["lr"] == {"type": "const", "val": 0.1}
    assert cfg["hyperparameters"]["opt"]["mom"]["type"] == "double"
