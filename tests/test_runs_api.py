"""Flat runs API + bulk experiment actions + experiment detail reads (reference api_runs.go
SearchRuns / MoveRuns, api_experiment.go bulk actions, GetExperimentValidationHistory,
ExpMetricNames, GetModelDefTree / GetModelDefFile) against an in-process master."""

import base64
import io
import tarfile

import pytest

from determined_amd.common.api import APIException, Session

CFG = {"name": "r", "hyperparameters": {}, "searcher": {"name": "single", "metric": "loss",
                                                       "smaller_is_better": True, "max_length": {"batches": 1}}}


@pytest.fixture()
def master():
    from determined_amd.master import start_master

    srv = start_master()
    yield srv, Session(f"http://127.0.0.1:{srv.port}")
    srv.stop()
    srv.master.close()


def _exp_with_trials(s, n, name="r"):
    eid = s.post("/api/v1/unmanaged/experiments", {"config": dict(CFG, name=name)})["experiment"]["id"]
    tids = [s.post(f"/api/v1/unmanaged/experiments/{eid}/trials", {"hparams": {"i": i}})["trial_id"] for i in range(n)]
    return eid, tids


def test_search_and_move_runs(master):
    srv, s = master
    e1, (t1, t2) = _exp_with_trials(s, 2, "two")
    e2, (t3,) = _exp_with_trials(s, 1, "one")
    got = s.post("/api/v1/runs", {})
    assert [r["id"] for r in got["runs"]] == [t1, t2, t3] and got["pagination"]["total"] == 3
    assert got["runs"][0]["experiment_name"] == "two" and got["runs"][0]["searcher_metric"] == "loss"
    assert [r["id"] for r in s.post("/api/v1/runs", {"sort": "id=desc", "limit": 2})["runs"]] == [t3, t2]
    assert [r["id"] for r in s.post("/api/v1/runs", {"experiment_ids": [e2]})["runs"]] == [t3]
    with pytest.raises(APIException):
        s.post("/api/v1/runs", {"sort": "bogus=asc"})
    ws = s.post("/api/v1/workspaces", {"name": "w"})["workspace"]
    proj = s.post(f"/api/v1/workspaces/{ws['id']}/projects", {"name": "p"})["project"]
    res = s.post("/api/v1/runs/move", {"run_ids": [t1, t3], "destination_project_id": proj["id"]})["results"]
    errs = {r["id"]: r["error"] for r in res}
    assert errs[t3] == "" and "other runs" in errs[t1]  # t1's experiment also has t2
    assert [r["id"] for r in s.post("/api/v1/runs", {"project_id": proj["id"]})["runs"]] == [t3]
    s.post("/api/v1/runs/move", {"run_ids": [t1, t2], "destination_project_id": proj["id"]})
    assert len(s.post("/api/v1/runs", {"project_id": proj["id"]})["runs"]) == 3


def test_bulk_actions_history_metric_names_and_files(master):
    srv, s = master
    e1, (t1,) = _exp_with_trials(s, 1)
    e2, (t2,) = _exp_with_trials(s, 1)
    for steps, loss in ((1, 3.0), (2, 4.0), (3, 2.0)):
        s.post(f"/api/v1/trials/{t1}/metrics", {"group": "validation", "steps_completed": steps,
                                               "metrics": {"loss": loss, "acc": 0.1}})
    s.post(f"/api/v1/trials/{t1}/metrics", {"group": "training", "steps_completed": 3, "metrics": {"loss": 1.0}})
    hist = s.get(f"/api/v1/experiments/{e1}/validation-history")["validation_history"]
    assert [h["searcher_metric"] for h in hist] == [3.0, 2.0]
    names = s.get(f"/api/v1/experiments/{e1}/metric-names")
    assert names["metric_names"] == {"training": ["loss"], "validation": ["acc", "loss"]}
    res = s.post("/api/v1/experiments/bulk/archive", {"experiment_ids": [e1, e2, 999]})["results"]
    assert [r["error"] == "" for r in res] == [True, True, False]
    assert s.post("/api/v1/runs", {"archived": True})["pagination"]["total"] == 2
    res = s.post("/api/v1/experiments/bulk/unarchive", {"filters": {"archived": True}})["results"]
    assert sorted(r["id"] for r in res) == [e1, e2]
    # model definition tree / file
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as tf:
        data = b"print('hi')\n"
        ti = tarfile.TarInfo("model_def.py")
        ti.size = len(data)
        tf.addfile(ti, io.BytesIO(data))
    eid = s.post("/api/v1/experiments", {"config": dict(CFG, entrypoint="model_def:T"), "activate": False,
                                         "model_def": base64.b64encode(buf.getvalue()).decode()})["experiment"]["id"]
    assert [f["path"] for f in s.get(f"/api/v1/experiments/{eid}/file_tree")["files"]] == ["model_def.py"]
    got = s.post(f"/api/v1/experiments/{eid}/file", {"path": "model_def.py"})["file"]
    assert base64.b64decode(got) == data
    with pytest.raises(APIException):
        s.post(f"/api/v1/experiments/{eid}/file", {"path": "nope.py"})
