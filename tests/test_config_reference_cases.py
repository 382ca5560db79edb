"""Replay the reference's expconf test corpus (schemas/test_cases/v0/*.yaml, read as data with
yaml.safe_load) against determined_amd.config._schema.

Each reference case holds a config under ``case`` and any of: ``sane_as`` (schemas it must pass),
``sanity_errors`` ({schema: [regex, ...]} -- every regex must match one rendered error),
``complete_as`` / ``completeness_errors`` (the same after eventually-required fields are enforced),
``default_as`` + ``defaulted`` (the config with defaults filled; ``"*"`` marks a runtime default that only
needs to be non-null), ``merge_as`` + ``merge_src`` + ``merged`` (template merging).
The reference runs the same corpus from Go (master/pkg/schemas/expconf/schema_test.go) and Python
(harness/tests/common/test_schemas.py)."""

import glob
import os
import re

import pytest
import yaml

from determined_amd.config import _schema as S

CASE_DIR = "/root/reference/schemas/test_cases/v0"
FILES = sorted(glob.glob(os.path.join(CASE_DIR, "*.yaml")))

# Cases whose expectations depend on behaviour this implementation intentionally does not reproduce.
SKIPS = {}


def _cases():
    out = []
    for f in FILES:
        with open(f) as fh:
            for c in yaml.safe_load(fh) or []:
                out.append(pytest.param(c, id=f"{os.path.basename(f)}::{c['name']}"))
    return out


def _name(url):
    return url.rsplit("/", 1)[-1]


def _clear_runtime_defaults(obj, expected):
    """Where the expectation says "*", a non-null value is accepted (and replaced by "*")."""
    if expected == "*":
        return "*" if obj is not None else obj
    if isinstance(obj, dict) and isinstance(expected, dict):
        return {k: _clear_runtime_defaults(v, expected.get(k)) if k in expected else v for k, v in obj.items()}
    if isinstance(obj, list) and isinstance(expected, list) and len(obj) == len(expected):
        return [_clear_runtime_defaults(a, b) for a, b in zip(obj, expected)]
    return obj


def _norm(v):
    """YAML floats vs ints: compare numbers by value."""
    if isinstance(v, dict):
        return {k: _norm(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_norm(x) for x in v]
    if isinstance(v, float) and v.is_integer():
        return int(v)
    return v


def _check_errors(errors, patterns, what):
    assert errors, f"expected {what} errors matching {patterns}, got none"
    for p in patterns:
        assert any(re.search(p, e) for e in errors), f"no {what} error matches {p!r}; got {errors}"


@pytest.mark.skipif(not FILES, reason="reference schema corpus not present")
@pytest.mark.parametrize("case", _cases())
def test_reference_case(case):
    if case["name"] in SKIPS:
        pytest.skip(SKIPS[case["name"]])
    value = case["case"]
    for url in case.get("sane_as") or []:
        errs = S.sanity_errors(value, _name(url))
        assert not errs, f"not sane as {_name(url)}: {errs}"
    for url, pats in (case.get("sanity_errors") or {}).items():
        _check_errors(S.sanity_errors(value, _name(url)), pats, "sanity")
    for url in case.get("complete_as") or []:
        errs = S.completeness_errors(value, _name(url))
        assert not errs, f"not complete as {_name(url)}: {errs}"
    for url, pats in (case.get("completeness_errors") or {}).items():
        _check_errors(S.completeness_errors(value, _name(url)), pats, "completeness")
    if case.get("default_as"):
        got = S.with_defaults(value, _name(case["default_as"]))
        exp = case["defaulted"]
        assert _norm(_clear_runtime_defaults(got, exp)) == _norm(exp)
    if case.get("merge_as"):
        got = S.merge(value, case["merge_src"], _name(case["merge_as"]))
        assert _norm(got) == _norm(case["merged"])


def test_corpus_coverage():
    """The corpus is replayed nearly whole: at most the documented SKIPS are left out."""
    if not FILES:
        pytest.skip("reference schema corpus not present")
    total = sum(len(yaml.safe_load(open(f)) or []) for f in FILES)
    assert total >= 130 and len(SKIPS) <= total - 120


def test_parse_rejects_unknown_keys_and_bad_types():
    from determined_amd import config as C

    base = {"searcher": {"name": "single", "metric": "loss", "max_length": {"batches": 10}}}
    C.parse(base)
    for bad, pat in [({**base, "bogus": 1}, "additional property 'bogus'"),
                     ({**base, "resources": {"slots_per_trail": 2}}, "slots_per_trail"),
                     ({**base, "searcher": {**base["searcher"], "max_length": {"batches": 1, "epochs": 2}}},
                      "length object"),
                     ({**base, "checkpoint_storage": {"type": "s3", "bucket": "b", "prefix": "a/../b"}}, "/../"),
                     ({**base, "profiling": {"begin_on_batch": 5, "end_after_batch": 2}}, "begin_on_batch")]:
        with pytest.raises(C.InvalidConfig) as ei:
            C.parse(bad)
        assert any(pat in e for e in ei.value.errors), ei.value.errors


def test_defaulted_config_is_sane():
    from determined_amd import config as C

    cfg = C.parse({"searcher": {"name": "adaptive_asha", "metric": "l", "max_trials": 4, "max_length": 100},
                   "hyperparameters": {"lr": 0.1, "n": {"b": {"type": "categorical", "vals": [1, 2]}}}})
    assert C.sanity_errors(cfg) == []
    assert S.completeness_errors(cfg) == []
