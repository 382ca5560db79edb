"""Resource pools (reference: master config ``resource_pools``, ``rm/agentrm/resource_pool.go``,
workspace bindings ``api_resourcepool.go``): per-pool schedulers, agents / trials / commands
landing in the right pool, defaults, job queues per pool, workspace bindings."""

import pytest

from determined_amd.common.api import APIException, Session

POOLS = [{"pool_name": "train", "scheduler": {"type": "fair_share"}},
         {"pool_name": "aux", "description": "notebooks", "scheduler": {"type": "round_robin"}}]
CFG = {"name": "p", "entrypoint": "model_def:T", "hyperparameters": {},
       "searcher": {"name": "single", "metric": "loss", "max_length": {"batches": 1}}}


@pytest.fixture()
def pooled():
    from determined_amd.master import start_master

    srv = start_master(resource_pools=POOLS, default_compute_pool="train", default_aux_pool="aux")
    yield srv, Session(f"http://127.0.0.1:{srv.port}")
    srv.stop()
    srv.master.close()


def _assigned(m, task_id):
    with m.lock:
        m._schedule()
        a = next(a for a in m.allocations.values() if a.task_id == task_id)
        return [ag for ag, _ in a.assignment]


def test_agents_and_tasks_land_in_their_pools(pooled):
    srv, s = pooled
    m = srv.master
    s.post("/api/v1/agents/register", {"agent_id": "gpu-node", "slots": 8, "resource_pool": "train"})
    s.post("/api/v1/agents/register", {"agent_id": "cpu-node", "slots": 2, "resource_pool": "aux"})
    with pytest.raises(APIException) as e:
        s.post("/api/v1/agents/register", {"agent_id": "x", "slots": 1, "resource_pool": "nope"})
    assert e.value.status == 400
    pools = {p["name"]: p for p in s.get("/api/v1/resource-pools")["resource_pools"]}
    assert pools["train"]["slots_available"] == 8 and pools["train"]["scheduler_type"] == "fair_share"
    assert pools["aux"]["slots_available"] == 2 and pools["aux"]["default_aux_pool"]
    assert {a["id"]: a["resource_pool"] for a in s.get("/api/v1/agents")["agents"]} == {"gpu-node": "train",
                                                                                      "cpu-node": "aux"}
    # slots > 0 -> default compute pool; 0 slots -> default aux pool; explicit pool wins
    t1 = s.post("/api/v1/commands", {"command": ["sleep", "1"], "slots": 4})["task_id"]
    t0 = s.post("/api/v1/commands", {"command": ["sleep", "1"], "slots": 0})["task_id"]
    t2 = s.post("/api/v1/commands", {"command": ["sleep", "1"], "slots": 1, "resource_pool": "aux"})["task_id"]
    assert _assigned(m, t1) == ["gpu-node"]
    assert _assigned(m, t2) == ["cpu-node"]
    jobs = s.get("/api/v1/job-queues", params={"resource_pool": "aux"})["jobs"]
    assert {j["job_id"] for j in jobs} == {t0, t2} and all(j["resource_pool"] == "aux" for j in jobs)
    # a request larger than its pool never spills into another pool
    big = s.post("/api/v1/commands", {"command": ["sleep", "1"], "slots": 3, "resource_pool": "aux"})["task_id"]
    assert _assigned(m, big) == []


def test_experiment_pool_validation_and_workspace_bindings(pooled):
    srv, s = pooled
    with pytest.raises(APIException) as e:
        s.post("/api/v1/experiments", {"config": dict(CFG, resources={"resource_pool": "nope"}), "activate": False})
    assert e.value.status == 400
    eid = s.post("/api/v1/experiments", {"config": CFG, "activate": False})["experiment"]["id"]
    assert srv.master.experiments[eid].config["resources"]["resource_pool"] == "train"
    ws = s.post("/api/v1/workspaces", {"name": "vision"})["workspace"]
    s.post(f"/api/v1/workspaces/{ws['id']}/projects", {"name": "detection"})
    got = s.request("PUT", "/api/v1/resource-pools/train/workspace-bindings", body={"workspace_names": ["vision"]})
    assert got["workspaces"] == ["vision"]
    assert s.get("/api/v1/resource-pools/train/workspace-bindings")["workspaces"] == ["vision"]
    with pytest.raises(APIException) as e:  # the Uncategorized workspace may no longer use "train"
        s.post("/api/v1/experiments", {"config": CFG, "activate": False})
    assert e.value.status == 400
    s.post("/api/v1/experiments", {"config": dict(CFG, workspace="vision", project="detection"), "activate": False})
    assert s.get("/api/v1/workspaces/Uncategorized/available-resource-pools")["resource_pools"] == ["aux"]
    assert sorted(s.get("/api/v1/workspaces/vision/available-resource-pools")["resource_pools"]) == ["aux", "train"]
    s.request("DELETE", "/api/v1/resource-pools/train/workspace-bindings", body={"workspace_names": ["vision"]})
    assert s.get("/api/v1/resource-pools/train/workspace-bindings")["workspaces"] == []


def test_single_default_pool_without_config():
    from determined_amd.master import start_master

    srv = start_master()
    try:
        s = Session(f"http://127.0.0.1:{srv.port}")
        (p,) = s.get("/api/v1/resource-pools")["resource_pools"]
        assert p["name"] == "default" and p["default_compute_pool"] and p["default_aux_pool"]
    finally:
        srv.stop()
        srv.master.close()


def test_sdk_resource_pool_and_determined_object(pooled):
    """SDK ``ResourcePool`` bindings + the object-style ``Determined`` client (reference
    ``common/experimental/{resource_pool,determined}.py``)."""
    from determined_amd.experimental import Determined, ResourcePool, client

    srv, s = pooled
    d = Determined(f"http://127.0.0.1:{srv.port}")
    assert sorted(p.name for p in d.list_resource_pools()) == ["aux", "train"]
    w = d.create_workspace("vision")
    w.create_project("detection")
    rp = d.get_resource_pool("train")
    assert isinstance(rp, ResourcePool) and rp.describe()["scheduler_type"] == "fair_share"
    rp.add_bindings(["vision"])
    assert rp.list_workspaces() == ["vision"]
    assert sorted(p.name for p in w.list_pools()) == ["aux", "train"]
    assert [p.name for p in d.get_workspace("Uncategorized").list_pools()] == ["aux"]
    rp.replace_bindings([])
    assert rp.list_workspaces() == []
    rp.add_bindings(["vision"])
    rp.remove_bindings(["vision"])
    assert rp.list_workspaces() == []
    exp = d.create_experiment(dict(CFG, workspace="vision", project="detection"), activate=False)
    assert [e.id for e in d.list_experiments()] == [exp.id]
    assert d.get_experiment(exp.id).config["resources"]["resource_pool"] == "train"
    # the object's session never leaks into the module-level client
    assert client._override.get() is None


def test_test_one_batch_runs_a_trial_locally(tmp_path, monkeypatch):
    """``experimental.test_one_batch`` (reference ``experimental/_native.py``): one training
    batch + validation + checkpoint of a PyTorchTrial in test mode."""
    import os
    import sys

    from determined_amd.experimental import test_one_batch

    monkeypatch.chdir(tmp_path)
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "fixtures", "tiny_trial"))
    try:
        from model_def import TinyTrial

        calls = []
        orig = TinyTrial.train_batch
        monkeypatch.setattr(TinyTrial, "train_batch", lambda self, *a, **k: calls.append(1) or orig(self, *a, **k))
        test_one_batch(TinyTrial, {"hyperparameters": {"global_batch_size": 8, "lr": 0.1}})
        assert len(calls) == 1
    finally:
        sys.path.pop(0)


def test_agent_restart_marks_lost_allocations(pooled):
    """An agent that re-registers without an allocation it was running (its process restarted:
    reference e2e test_agent_restart without reattach) gets that allocation failed, so trials
    restart under max_restarts instead of hanging; a plain reconnect listing it changes nothing."""
    srv, s = pooled
    m = srv.master
    s.post("/api/v1/agents/register", {"agent_id": "n", "slots": 8, "resource_pool": "train"})
    t1 = s.post("/api/v1/commands", {"command": ["sleep", "60"], "slots": 1})["task_id"]
    t2 = s.post("/api/v1/commands", {"command": ["sleep", "60"], "slots": 1})["task_id"]
    with m.lock:
        m._schedule()
    a1, a2 = (next(a for a in m.allocations.values() if a.task_id == t) for t in (t1, t2))
    assert len(s.get("/api/v1/agents/n/work", params={"timeout_seconds": 0})["commands"]) == 2
    for a in (a1, a2):
        s.post("/api/v1/agents/n/events", {"type": "started", "allocation_id": a.id})
    s.post("/api/v1/agents/register", {"agent_id": "n", "slots": 8, "resource_pool": "train", "running": [a1.id, a2.id]})
    assert a1.state == "RUNNING" and a2.state == "RUNNING"
    s.post("/api/v1/agents/register", {"agent_id": "n", "slots": 8, "resource_pool": "train", "running": [a2.id]})
    assert a1.state == "TERMINATED" and a2.state == "RUNNING"
    assert s.get(f"/api/v1/tasks/{t1}")["task"]["exit_code"] == -1


def test_agent_restart_loses_assigned_allocations_too(pooled):
    """an agent that pulled a start command and died before reporting 'started' (the
    allocation is ASSIGNED, no longer queued) has that allocation failed on re-registration; one
    still queued for it, or listed by the agent, is kept."""
    srv, s = pooled
    m = srv.master
    s.post("/api/v1/agents/register", {"agent_id": "n2", "slots": 8, "resource_pool": "train"})
    t1 = s.post("/api/v1/commands", {"command": ["sleep", "60"], "slots": 1})["task_id"]
    with m.lock:
        m._schedule()
    a1 = next(a for a in m.allocations.values() if a.task_id == t1)
    assert a1.state == "ASSIGNED"
    # the agent listing it as running (its start command just arrived) keeps it
    assert len(s.get("/api/v1/agents/n2/work", params={"timeout_seconds": 0})["commands"]) == 1
    s.post("/api/v1/agents/register", {"agent_id": "n2", "slots": 8, "resource_pool": "train", "running": [a1.id]})
    assert a1.state == "ASSIGNED"
    # a restarted agent (empty list) lost it
    s.post("/api/v1/agents/register", {"agent_id": "n2", "slots": 8, "resource_pool": "train", "running": []})
    assert a1.state == "TERMINATED"
    assert s.get(f"/api/v1/tasks/{t1}")["task"]["exit_code"] == -1


def test_agent_reregistering_into_another_pool_moves_its_slots(pooled):
    """a known agent re-registering with another --resource-pool (or slot count) is
    rebuilt in the scheduler: its slots count in the new pool, work lands there, and allocations it
    held through the old pool are failed as lost."""
    srv, s = pooled
    m = srv.master
    s.post("/api/v1/agents/register", {"agent_id": "mv", "slots": 4, "resource_pool": "train"})
    t1 = s.post("/api/v1/commands", {"command": ["sleep", "60"], "slots": 1, "resource_pool": "train"})["task_id"]
    assert _assigned(m, t1) == ["mv"]
    a1 = next(a for a in m.allocations.values() if a.task_id == t1)
    s.post("/api/v1/agents/register", {"agent_id": "mv", "slots": 2, "resource_pool": "aux", "running": [a1.id]})
    assert a1.state == "TERMINATED"
    pools = {p["name"]: p for p in s.get("/api/v1/resource-pools")["resource_pools"]}
    assert pools["train"]["slots_available"] == 0 and pools["aux"]["slots_available"] == 2
    assert {a["id"]: a["resource_pool"] for a in s.get("/api/v1/agents")["agents"]} == {"mv": "aux"}
    # new work for the aux pool lands on it; the train pool has nothing left to offer
    t2 = s.post("/api/v1/commands", {"command": ["sleep", "1"], "slots": 1, "resource_pool": "aux"})["task_id"]
    t3 = s.post("/api/v1/commands", {"command": ["sleep", "1"], "slots": 1, "resource_pool": "train"})["task_id"]
    assert _assigned(m, t2) == ["mv"] and _assigned(m, t3) == []
