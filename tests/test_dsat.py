"""DeepSpeed autotuning: search-method logic against simulated outcomes, and an end-to-end
binary search over a CPU cluster (in-process master + agent running real trial processes)
where micro-batches above 12 "run out of memory" (reference tests:
``harness/tests/experiment/pytorch/test_dsat.py``)."""

import json
import pathlib
import tempfile
import threading
import uuid

import pytest

from determined_amd.pytorch.dsat import BinarySearchDSATSearchMethod, RandomDSATSearchMethod, candidate_hparams
from determined_amd.pytorch.dsat._search import Candidate
from determined_amd.searcher import Create, ExitedReason, SearcherState, Shutdown

ROOT = pathlib.Path(__file__).resolve().parent.parent
FIX = ROOT / "tests" / "fixtures" / "dsat_trial"


def _simulate(method, fits, tput):
    """Drive a search method with a fake cluster: mbs > fits[stage] OOMs, else tput(stage, mbs)."""
    st = SearcherState()
    pending = [op for op in method.initial_operations(st) if isinstance(op, Create)]
    shut = False
    n = 0
    while pending and n < 200:
        n += 1
        op = pending.pop(0)
        c = method.trials[str(op.request_id)]
        hp = op.hparams
        assert hp["overwrite_deepspeed_args"]["zero_optimization"]["stage"] == c.stage
        assert hp["overwrite_deepspeed_args"]["train_micro_batch_size_per_gpu"] == c.mbs
        assert hp["_dsat_mode"]["end_profile_step"] == method.end
        if c.mbs > fits[c.stage]:
            ops = method.on_trial_exited_early(st, op.request_id, ExitedReason.INVALID_HP)
        else:
            method.on_validation_completed(st, op.request_id, tput(c.stage, c.mbs), method.end)
            ops = method.on_trial_closed(st, op.request_id)
        pending += [o for o in ops if isinstance(o, Create)]
        shut = shut or any(isinstance(o, Shutdown) for o in ops)
    return shut


def test_binary_search_finds_largest_fitting_mbs_per_stage():
    m = BinarySearchDSATSearchMethod({}, [1, 2, 3], max_trials=64, max_concurrent=3, max_mbs=64)
    fits = {1: 9, 2: 17, 3: 40}
    assert _simulate(m, fits, lambda s, b: b * (1.0 + 0.1 * s))
    ok = {}
    for c in m.trials.values():
        if not c.oom:
            ok[c.stage] = max(ok.get(c.stage, 0), c.mbs)
    assert ok == fits
    best = m.best()
    assert (best.stage, best.mbs) == (3, 40)
    # every probe of a stage is a distinct micro-batch and the search is logarithmic
    assert len(m.trials) <= 3 * 7


def test_random_search_prunes_after_oom_and_latency_metric():
    m = RandomDSATSearchMethod({}, [2], max_trials=12, max_concurrent=2, max_mbs=32, metric="latency")
    _simulate(m, {2: 10}, lambda s, b: 1.0 / b)
    assert all(c.mbs <= 10 or c.oom for c in m.trials.values())
    assert m.best().mbs <= 10 and m.smaller_is_better


def test_candidate_hparams_merge():
    hp = candidate_hparams({"overwrite_deepspeed_args": {"gradient_clipping": 1.0, "train_batch_size": 64,
                                                         "zero_optimization": {"overlap_comm": True}}, "lr": 3},
                           Candidate(2, 8), 3, 5, "throughput")
    ow = hp["overwrite_deepspeed_args"]
    assert ow == {"gradient_clipping": 1.0, "train_micro_batch_size_per_gpu": 8,
                  "zero_optimization": {"overlap_comm": True, "stage": 2}}
    assert hp["lr"] == 3 and hp["_dsat_mode"]["start_profile_step"] == 3


@pytest.fixture(scope="module")
def cluster():
    from determined_amd.agent import Agent
    from determined_amd.common.api import Session
    from determined_amd.master import start_master

    srv = start_master()
    url = f"http://127.0.0.1:{srv.port}"
    ag = Agent(url, "dsat-agent", slots=4, work_root=tempfile.mkdtemp())
    threading.Thread(target=ag.run, daemon=True).start()
    yield {"url": url, "s": Session(url)}
    ag.stop()
    srv.stop()


def test_dsat_binary_e2e_on_cluster(cluster, tmp_path):
    import yaml

    from determined_amd.pytorch.dsat import run_autotuning

    cfg = yaml.safe_load((FIX / "dsat.yaml").read_text())
    cfg["checkpoint_storage"] = {"type": "shared_fs", "host_path": str(tmp_path / "ckpt")}
    cfg_path = tmp_path / "dsat.yaml"
    cfg_path.write_text(yaml.safe_dump(cfg))
    summary = run_autotuning("binary", str(cfg_path), str(FIX), session=cluster["s"],
                             searcher_dir=str(tmp_path / "state"), zero_stages=[1, 2], max_mbs=16,
                             max_trials=16, max_concurrent_trials=4, start_profile_step=1, end_profile_step=3,
                             run_full_experiment=True)
    trials = summary["trials"]
    assert {t["stage"] for t in trials} == {1, 2}
    assert any(t["oom"] for t in trials) and all(t["oom"] == (t["mbs"] > 12) for t in trials)
    best = summary["best"]
    assert best is not None and best["mbs"] <= 12 and best["metric"] > 0
    assert summary["best_hyperparameters"]["overwrite_deepspeed_args"]["zero_optimization"]["stage"] == best["stage"]
    exp = cluster["s"].get(f"/api/v1/experiments/{summary['search_experiment_id']}")["experiment"]
    assert exp["state"] == "COMPLETED"
    assert "full_experiment_id" in summary
    assert json.loads((tmp_path / "state" / "dsat_summary.json").read_text())["best"] == best
