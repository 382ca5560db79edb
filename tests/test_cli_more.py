"""The remaining reference ``det`` verbs (cli/_more.py) against an in-process master: agents,
master config, resource pools + bindings, resources accounting, user groups + group roles,
user rename/edit/link-with-agent-user, workspace/project extras, task/template extras,
preview-search, version, dev curl."""

import contextlib
import io
import json
import time

import pytest
import yaml

from determined_amd.common.api import Session


@pytest.fixture()
def master():
    from determined_amd.master import start_master

    srv = start_master(resource_pools=[{"pool_name": "default"}, {"pool_name": "aux"}], default_aux_pool="aux")
    yield srv, f"http://127.0.0.1:{srv.port}"
    srv.stop()
    srv.master.close()


def det(url, *args):
    from determined_amd.cli import main

    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        rc = main(["-m", url, *args])
    assert rc in (0, None), out.getvalue()
    return out.getvalue()


def test_cluster_and_admin_verbs(master, tmp_path):
    srv, url = master
    s = Session(url)
    s.post("/api/v1/agents/register", {"agent_id": "n1", "slots": 2})
    det(url, "agent", "disable", "n1")
    assert not s.get("/api/v1/agents")["agents"][0]["enabled"]
    det(url, "agent", "enable", "n1")
    det(url, "slot", "disable", "n1", "1")
    ag = s.get("/api/v1/agents")["agents"][0]
    assert ag["disabled_slots"] == [1]
    rows = json.loads(det(url, "--json", "slot", "list"))
    assert [r["enabled"] for r in rows] == [True, False]
    s.post("/api/v1/agents/register", {"agent_id": "n1", "slots": 2})  # re-registration keeps it
    assert s.get("/api/v1/agents")["agents"][0]["disabled_slots"] == [1]
    det(url, "slot", "enable", "n1", "1")
    assert s.get("/api/v1/agents")["agents"][0]["disabled_slots"] == []
    assert "resource_pools" in det(url, "master", "config", "show")
    assert "log level: debug" in det(url, "master", "config", "set", "--log-level", "debug")
    det(url, "master", "config", "set", "--log-level", "info")
    # pools + bindings
    det(url, "workspace", "create", "vision")
    det(url, "resource-pool", "bindings", "add", "aux", "vision")
    assert det(url, "resource-pool", "bindings", "list-workspaces", "aux").split() == ["vision"]
    assert det(url, "workspace", "list-pools", "Uncategorized").split() == ["default"]
    det(url, "resource-pool", "bindings", "remove", "aux", "vision")
    # commands: pool / priority / config / set priority / job update
    tid = s.post("/api/v1/commands", {"command": ["sleep", "5"], "slots": 1, "priority": 30})["task_id"]
    assert "priority: 30" in det(url, "cmd", "config", tid)
    det(url, "cmd", "set", "priority", tid, "7")
    job = next(j for j in s.get("/api/v1/job-queues")["jobs"] if j["job_id"] == tid)
    assert job["priority"] == 7
    det(url, "job", "update", tid, "--priority", "9")
    assert next(j for j in s.get("/api/v1/job-queues")["jobs"] if j["job_id"] == tid)["priority"] == 9
    # resources accounting (the command got the agent's slots)
    with srv.master.lock:
        srv.master._schedule()
    time.sleep(0.05)
    raw = json.loads(det(url, "resources", "raw", "0", str(time.time() + 5), "--json"))
    assert any(r["task_id"] == tid and r["slots"] == 1 and r["resource_pool"] == "default" for r in raw)
    today = time.strftime("%Y-%m-%d")
    agg = json.loads(det(url, "resources", "aggregated", today, today, "--json"))
    assert agg[0]["by_kind"]["COMMAND"] > 0
    det(url, "cmd", "kill", tid)
    # templates
    f = tmp_path / "t.yaml"
    f.write_text(yaml.safe_dump({"resources": {"slots_per_trial": 2}, "max_restarts": 1}))
    det(url, "template", "create", "base", str(f))
    f.write_text(yaml.safe_dump({"resources": {"priority": 5}}))
    det(url, "template", "set-value", "config", "base", str(f))
    got = s.get("/api/v1/templates/base")["template"]["config"]
    assert got["resources"] == {"slots_per_trial": 2, "priority": 5} and got["max_restarts"] == 1
    # tasks
    f.write_text(yaml.safe_dump({"entrypoint": ["true"], "resources": {"slots": 0}}))
    new = det(url, "task", "create", str(f)).split()[-1]
    assert s.get(f"/api/v1/tasks/{new}")["task"]["config"]["resource_pool"] == "aux"
    forked = det(url, "task", "fork", new).split()[-1]
    assert forked != new and s.get(f"/api/v1/tasks/{forked}")["task"]["config"]["cmd"] == ["true"]
    assert "removed" in det(url, "task", "cleanup-logs")
    assert "client:" in det(url, "version")
    assert json.loads(det(url, "dev", "curl", "/api/v1/me"))["user"]["username"] == "determined"


def test_users_groups_and_projects(master):
    srv, url = master
    det(url, "user", "create", "carol")
    det(url, "user", "rename", "carol", "caroline")
    det(url, "user", "edit", "caroline", "--display-name", "Caro")
    det(url, "user", "link-with-agent-user", "caroline", "--agent-uid", "1234", "--agent-gid", "1234",
        "--agent-user", "caro", "--agent-group", "ml")
    u = Session(url).get("/api/v1/users/caroline")["user"]
    assert u["display_name"] == "Caro" and u["agent_user_group"]["agent_uid"] == 1234
    det(url, "user-group", "create", "ml-team", "--add-user", "caroline")
    det(url, "user-group", "add-user", "ml-team", "determined")
    assert "caroline, determined" in det(url, "user-group", "describe", "ml-team")
    det(url, "user-group", "remove-user", "ml-team", "determined")
    det(url, "user-group", "change-name", "ml-team", "vision-team")
    assert "vision-team" in det(url, "user-group", "list", "--groups-user-belongs-to", "caroline")
    det(url, "workspace", "create", "ws1")
    det(url, "rbac", "assign-role", "Editor", "--group-name-to-assign", "vision-team", "--workspace-name", "ws1")
    assert "vision-team" in det(url, "rbac", "list-groups-roles")
    assert "edit" in det(url, "rbac", "describe-role", "Editor")
    assert "cluster" in det(url, "rbac", "my-permissions")
    det(url, "user-group", "delete", "vision-team")
    det(url, "project", "create", "ws1", "p1")
    det(url, "project", "edit", "ws1", "p1", "--description", "first")
    assert "p1" in det(url, "workspace", "list-projects", "ws1")
    det(url, "project", "list-experiments", "ws1", "p1")
    det(url, "workspace", "edit", "ws1", "--name", "ws2")
    assert "ws2" in det(url, "workspace", "list")


def test_group_roles_grant_permissions():
    """A role given to a group applies to its members (rbac mode)."""
    from determined_amd.master import start_master

    srv = start_master(auth="rbac")
    try:
        url = f"http://127.0.0.1:{srv.port}"
        admin = Session(url, token=Session(url).post("/api/v1/auth/login", {"username": "admin"})["token"])
        admin.post("/api/v1/users", {"username": "dave", "password": "pw"})
        ws = admin.post("/api/v1/workspaces", {"name": "team"})["workspace"]
        dave = Session(url, token=Session(url).post("/api/v1/auth/login",
                                                      {"username": "dave", "password": "pw"})["token"])
        with pytest.raises(Exception):
            dave.post(f"/api/v1/workspaces/{ws['id']}/projects", {"name": "x"})
        admin.post("/api/v1/groups", {"name": "g", "add_users": ["dave"]})
        admin.post("/api/v1/rbac/assign-group", {"group": "g", "role": "Editor", "workspace": "team"})
        dave.post(f"/api/v1/workspaces/{ws['id']}/projects", {"name": "x"})
        perms = dave.get("/api/v1/rbac/my-permissions")["permissions"]
        assert "edit" in perms["team"] and "edit" not in perms["cluster"]
    finally:
        srv.stop()
        srv.master.close()


def test_preview_search(tmp_path):
    from determined_amd.cli import main

    f = tmp_path / "c.yaml"
    f.write_text(yaml.safe_dump({
        "name": "p", "entrypoint": "x:T",
        "hyperparameters": {"lr": {"type": "log", "base": 10, "minval": -4, "maxval": -1}},
        "searcher": {"name": "adaptive_asha", "metric": "loss", "max_trials": 16, "max_length": {"batches": 1000},
                     "max_rungs": 3, "divisor": 4, "mode": "standard"}}))
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        main(["preview-search", str(f)])
    text = out.getvalue()
    assert "adaptive_asha" in text and "16 trial(s)" in text and "batches" in text


def test_experiment_create_template_project_and_includes(master, tmp_path):
    """``det e create --template/--project_id/-i`` (reference cli/experiment.py + core_experiment.go
    ``schemas.Merge(config, template)``: the experiment's own settings win) and ``det cmd run
    --template``."""
    import base64
    import io
    import tarfile

    srv, url = master
    s = Session(url)
    tpl = tmp_path / "tpl.yaml"
    tpl.write_text(yaml.safe_dump({"max_restarts": 7, "resources": {"slots_per_trial": 2, "priority": 11},
                                   "environment": {"environment_variables": ["FROM_TPL=1"]}}))
    det(url, "template", "create", "team", str(tpl))
    cfg = tmp_path / "exp.yaml"
    cfg.write_text(yaml.safe_dump({"name": "tpl", "entrypoint": "model_def:T", "hyperparameters": {},
                                   "resources": {"slots_per_trial": 1},
                                   "searcher": {"name": "single", "metric": "loss", "max_length": {"batches": 1}}}))
    model = tmp_path / "model"
    model.mkdir()
    (model / "model_def.py").write_text("T = None\n")
    extra = tmp_path / "extra.txt"
    extra.write_text("hello")
    det(url, "workspace", "create", "ws")
    det(url, "project", "create", "ws", "proj")
    pid = next(p["id"] for p in s.get("/api/v1/workspaces/ws/projects")["projects"] if p["name"] == "proj")
    out = det(url, "experiment", "create", str(cfg), str(model), "--paused", "--template", "team",
              "--project_id", str(pid), "-i", str(extra))
    eid = int(out.split()[-1])
    exp = srv.master.experiments[eid]
    assert exp.config["max_restarts"] == 7  # from the template
    assert exp.config["resources"]["slots_per_trial"] == 1  # the experiment's own value wins
    assert exp.config["resources"]["priority"] == 11
    row = s.get(f"/api/v1/experiments/{eid}")["experiment"]
    assert (row.get("workspace"), row.get("project")) == ("ws", "proj")
    md = srv.master.db.one("SELECT model_def FROM experiments WHERE id=?", [eid])["model_def"]
    names = tarfile.open(fileobj=io.BytesIO(md if isinstance(md, bytes) else base64.b64decode(md))).getnames()
    assert {"model_def.py", "extra.txt"} <= set(names)
    with pytest.raises(AssertionError):  # the CLI exits non-zero: template not found
        det(url, "experiment", "create", str(cfg), str(model), "--paused", "--template", "nope")
    # commands: slots / priority / env from the template
    det(url, "cmd", "run", "-d", "--template", "team", "true")
    job = [j for j in s.get("/api/v1/job-queues")["jobs"] if j["job_id"].startswith("command-")][-1]
    assert job["priority"] == 11


def test_task_pause_unpause_dev_bindings_template_config(master, tmp_path):
    """``det task pause/unpause`` (reference api_generic_tasks.go: the allocation ends, the task
    waits in PAUSED, unpause starts it again), ``det dev bindings list/call``, ``det template
    config`` and ``det notebook open``."""
    srv, url = master
    s = Session(url)
    s.post("/api/v1/agents/register", {"agent_id": "n1", "slots": 2})
    tid = s.post("/api/v1/commands", {"command": ["sleep", "30"], "slots": 1, "type": "GENERIC"})["task_id"]
    with srv.master.lock:
        srv.master._schedule()
    det(url, "task", "pause", tid)
    alloc = next(a for a in srv.master.allocations.values() if a.task_id == tid)
    with srv.master.lock:  # the agent reports the killed process
        alloc.exit_codes = {0: -15}
        srv.master._finish_allocation(alloc)
    assert s.get(f"/api/v1/tasks/{tid}")["task"]["state"] == "PAUSED"
    with pytest.raises(AssertionError):
        det(url, "task", "pause", tid)  # already paused
    det(url, "task", "unpause", tid)
    assert s.get(f"/api/v1/tasks/{tid}")["task"]["state"] in ("PENDING", "RUNNING")
    allocs = [a for a in srv.master.allocations.values() if a.task_id == tid]
    assert len(allocs) == 2 and allocs[-1].command == ["sleep", "30"]
    det(url, "cmd", "kill", tid)
    out = det(url, "dev", "bindings", "list")
    assert "POST   /api/v1/tasks/([^/]+)/(pause|unpause)" in out and "GET    /api/v1/agents" in out
    assert json.loads(det(url, "dev", "bindings", "call", "GET", "/api/v1/agents"))["agents"][0]["id"] == "n1"
    f = tmp_path / "t.yaml"
    f.write_text(yaml.safe_dump({"resources": {"slots_per_trial": 2}}))
    det(url, "template", "create", "tc", str(f))
    f.write_text(yaml.safe_dump({"max_restarts": 3}))
    det(url, "template", "config", "tc", str(f))
    assert s.get("/api/v1/templates/tc")["template"]["config"] == {"resources": {"slots_per_trial": 2}, "max_restarts": 3}
    assert det(url, "notebook", "open", tid).strip() == "not ready"
