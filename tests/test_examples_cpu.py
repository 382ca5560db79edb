"""The shipped examples run end to end on a CPU cluster (in-process master + agent running real
trial processes), shrunk to seconds: CIFAR-10 adaptive ASHA (BASELINE config #3), the Core API
script under an adaptive search and under the torch_distributed launcher (2 gloo ranks)."""

import base64
import copy
import pathlib

import pytest
import yaml

from tests.test_e2e_cpu import _trials, _wait, cluster  # noqa: F401  (fixture)

ROOT = pathlib.Path(__file__).resolve().parent.parent


def _submit(cl, example: str, cfg_name: str, patch):
    from determined_amd.cli import tar_model_dir

    d = ROOT / "examples" / example
    cfg = yaml.safe_load((d / cfg_name).read_text())
    patch(cfg)
    cfg["checkpoint_storage"] = {"type": "shared_fs", "host_path": cl["ckpt"]}
    r = cl["session"].post("/api/v1/experiments", {"config": cfg, "activate": True,
                                                   "model_def": base64.b64encode(tar_model_dir(str(d))).decode()})
    return r["experiment"]["id"]


def test_cifar10_adaptive_asha_example(cluster):  # noqa: F811
    def shrink(cfg):
        cfg["searcher"].update(max_trials=4, max_concurrent_trials=2, max_length={"epochs": 2}, max_rungs=2)
        cfg["records_per_epoch"] = 256
        cfg["data"] = {"train_size": 256, "val_size": 64}
        cfg["hyperparameters"]["global_batch_size"] = 64

    eid = _submit(cluster, "cifar10_pytorch", "adaptive.yaml", shrink)
    e = _wait(cluster, eid, timeout=600)
    assert e["state"] == "COMPLETED"
    ts = _trials(cluster, eid)
    assert len(ts) == 4 and all(t["state"] == "COMPLETED" for t in ts)


def test_core_api_example_hpsearch_and_distributed(cluster):  # noqa: F811
    def small_search(cfg):
        cfg["searcher"].update(max_trials=2, max_concurrent_trials=2, max_length=100)

    eid = _submit(cluster, "core_api", "hpsearch.yaml", small_search)
    s = cluster["session"]
    if _wait(cluster, eid, timeout=600)["state"] != "COMPLETED":
        for t in _trials(cluster, eid):
            print("\n".join(l["log"] for l in s.get(f"/api/v1/tasks/trial-{t['id']}/logs")["logs"][-30:]))
        raise AssertionError("core_api hpsearch experiment did not complete")
    for t in _trials(cluster, eid):
        assert t["state"] == "COMPLETED"
        ms = s.get(f"/api/v1/trials/{t['id']}/metrics")
        assert "validation_loss" in str(ms)

    def small_dist(cfg):
        cfg["searcher"]["max_length"] = 100

    eid = _submit(cluster, "core_api", "distributed.yaml", small_dist)
    if _wait(cluster, eid, timeout=600)["state"] != "COMPLETED":
        for t in _trials(cluster, eid):
            print("\n".join(l["log"] for l in s.get(f"/api/v1/tasks/trial-{t['id']}/logs")["logs"][-200:]))
        raise AssertionError("core_api distributed experiment did not complete")
    (t,) = _trials(cluster, eid)
    logs = "\n".join(l["log"] for l in s.get(f"/api/v1/tasks/trial-{t['id']}/logs")["logs"])
    assert "[rank=1]" in logs  # both ranks ran under the launcher


def test_torch_batch_process_example(cluster):  # noqa: F811
    def small(cfg):
        pass

    eid = _submit(cluster, "torch_batch_process", "distributed.yaml", small)
    s = cluster["session"]
    if _wait(cluster, eid, timeout=600)["state"] != "COMPLETED":
        for t in _trials(cluster, eid):
            print("\n".join(l["log"] for l in s.get(f"/api/v1/tasks/trial-{t['id']}/logs")["logs"][-200:]))
        raise AssertionError("torch_batch_process example did not complete")
    (t,) = _trials(cluster, eid)
    ms = str(s.get(f"/api/v1/trials/{t['id']}/metrics"))
    assert "accuracy" in ms
    outs = list(pathlib.Path(cluster["ckpt"]).rglob("predictions_rank*.jsonl"))
    assert {p.name for p in outs} >= {"predictions_rank0.jsonl", "predictions_rank1.jsonl"}
    n = sum(len(p.read_text().splitlines()) for p in outs)
    assert n == 1024


def test_unmanaged_example(cluster, tmp_path):  # noqa: F811
    import os
    import subprocess
    import sys

    env = dict(os.environ, DET_MASTER=cluster["url"], DET_UNMANAGED_STORAGE=str(tmp_path),
               PYTHONPATH=str(ROOT), EXTERNAL_EXP_ID="ex-unmanaged-test")
    r = subprocess.run([sys.executable, str(ROOT / "examples" / "unmanaged" / "train.py")], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    s = cluster["session"]
    exps = [e for e in s.get("/api/v1/experiments")["experiments"] if e["name"] == "unmanaged-example"]
    assert exps and exps[-1]["unmanaged"]
    (t,) = _trials(cluster, exps[-1]["id"])
    assert "validation_loss" in str(s.get(f"/api/v1/trials/{t['id']}/metrics"))
    assert s.get(f"/api/v1/experiments/{exps[-1]['id']}/checkpoints")["checkpoints"]
