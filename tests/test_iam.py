"""Users, sessions, workspaces/projects and RBAC on an in-process master (reference tests:
``master/internal/user/*_test.go``, ``rbac`` authz tests, e2e ``test_workspace_org.py``)."""

import os

import pytest

from determined_amd.common.api import APIException, Session

CFG = {"name": "iam", "entrypoint": "model_def:T", "searcher": {"name": "single", "metric": "loss",
                                                                "max_length": {"batches": 1}},
       "hyperparameters": {}, "resources": {"slots_per_trial": 1}}


@pytest.fixture(scope="module")
def rbac_master():
    from determined_amd.master import start_master

    srv = start_master(auth="rbac", auth_token="cluster-secret")
    yield f"http://127.0.0.1:{srv.port}", srv.master
    srv.stop()
    srv.master.close()


def _login(url, user, pw=""):
    tok = Session(url).post("/api/v1/auth/login", {"username": user, "password": pw})["token"]
    return Session(url, token=tok)


def _exp_cfg(ws="Uncategorized", proj="Uncategorized"):
    return dict(CFG, workspace=ws, project=proj)


def test_auth_required_and_login(rbac_master):
    url, _ = rbac_master
    with pytest.raises(APIException) as e:
        Session(url).get("/api/v1/experiments")
    assert e.value.status == 401
    with pytest.raises(APIException) as e:
        Session(url).post("/api/v1/auth/login", {"username": "admin", "password": "wrong"})
    assert e.value.status == 401
    admin = _login(url, "admin")
    assert admin.get("/api/v1/me")["user"] == {"id": 1, "username": "admin", "display_name": "", "admin": True,
                                                "active": True}
    # the cluster token (agents/tasks) is accepted as the internal identity
    assert Session(url, token="cluster-secret").get("/api/v1/me")["user"]["admin"]
    admin.post("/api/v1/auth/logout", {})
    with pytest.raises(APIException):
        admin.get("/api/v1/me")


def test_users_workspaces_roles(rbac_master):
    url, m = rbac_master
    admin = _login(url, "admin")
    admin.post("/api/v1/users", {"username": "alice", "password": "pw1"})
    admin.post("/api/v1/users", {"username": "bob", "password": "pw2"})
    with pytest.raises(APIException) as e:
        admin.post("/api/v1/users", {"username": "alice"})
    assert e.value.status == 409
    alice = _login(url, "alice", "pw1")
    bob = _login(url, "bob", "pw2")
    with pytest.raises(APIException) as e:
        alice.post("/api/v1/users", {"username": "mallory"})
    assert e.value.status == 403

    ws = admin.post("/api/v1/workspaces", {"name": "vision"})["workspace"]
    proj = admin.post("/api/v1/workspaces/vision/projects", {"name": "resnet"})["project"]
    # no role in 'vision': cannot create an experiment there
    with pytest.raises(APIException) as e:
        alice.post("/api/v1/experiments", {"config": _exp_cfg("vision", "resnet"), "activate": False})
    assert e.value.status == 403
    admin.post("/api/v1/rbac/assign", {"user": "alice", "role": "Editor", "workspace": "vision"})
    admin.post("/api/v1/rbac/assign", {"user": "bob", "role": "Viewer", "workspace": "vision"})
    eid = alice.post("/api/v1/experiments", {"config": _exp_cfg("vision", "resnet"),
                                             "activate": False})["experiment"]["id"]
    exp = bob.get(f"/api/v1/experiments/{eid}")["experiment"]
    assert exp["owner"] == "alice" and exp["workspace"] == "vision" and exp["project"] == "resnet"
    with pytest.raises(APIException) as e:  # viewer cannot kill
        bob.post(f"/api/v1/experiments/{eid}/kill", {})
    assert e.value.status == 403
    # scoped role does not leak into other workspaces
    admin.post("/api/v1/workspaces", {"name": "nlp"})
    admin.post("/api/v1/workspaces/nlp/projects", {"name": "bert"})
    with pytest.raises(APIException):
        alice.post("/api/v1/experiments", {"config": _exp_cfg("nlp", "bert"), "activate": False})
    roles = {(r["username"], r["role"], r["workspace"]) for r in admin.get("/api/v1/rbac/assignments")["assignments"]}
    assert ("alice", "Editor", "vision") in roles and ("bob", "Viewer", "vision") in roles
    # projects: listing counts experiments; move between projects needs edit on both sides
    lst = alice.get(f"/api/v1/workspaces/{ws['id']}/projects")["projects"]
    assert [p["num_experiments"] for p in lst if p["name"] == "resnet"] == [1]
    other = admin.post("/api/v1/workspaces/vision/projects", {"name": "vit"})["project"]
    alice.post(f"/api/v1/experiments/{eid}/move", {"destination_project_id": other["id"]})
    assert alice.get(f"/api/v1/experiments/{eid}")["experiment"]["project"] == "vit"
    nlp_bert = [p for p in admin.get("/api/v1/workspaces/nlp/projects")["projects"]][0]
    with pytest.raises(APIException):
        alice.post(f"/api/v1/experiments/{eid}/move", {"destination_project_id": nlp_bert["id"]})
    # archived project refuses new experiments; a workspace holding experiments cannot be deleted
    admin.post(f"/api/v1/projects/{proj['id']}/archive", {})
    with pytest.raises(APIException) as e:
        alice.post("/api/v1/experiments", {"config": _exp_cfg("vision", "resnet"), "activate": False})
    assert e.value.status == 400
    with pytest.raises(APIException) as e:
        admin.delete("/api/v1/workspaces/vision")
    assert e.value.status == 409
    # deactivated users cannot log in; password change invalidates sessions
    admin.patch("/api/v1/users/bob", {"active": False})
    with pytest.raises(APIException):
        _login(url, "bob", "pw2")
    alice.post("/api/v1/users/alice/password", {"password": "new"})
    with pytest.raises(APIException):
        alice.get("/api/v1/me")
    assert _login(url, "alice", "new").get("/api/v1/me")["user"]["username"] == "alice"


def test_basic_mode_owner_rules():
    from determined_amd.master import start_master

    srv = start_master(auth="basic")
    url = f"http://127.0.0.1:{srv.port}"
    try:
        admin = _login(url, "admin")
        admin.post("/api/v1/users", {"username": "carol", "password": "x"})
        admin.post("/api/v1/users", {"username": "dave", "password": "y"})
        carol, dave = _login(url, "carol", "x"), _login(url, "dave", "y")
        eid = carol.post("/api/v1/experiments", {"config": _exp_cfg(), "activate": False})["experiment"]["id"]
        assert dave.get(f"/api/v1/experiments/{eid}")["experiment"]["owner"] == "carol"  # view: everyone
        with pytest.raises(APIException) as e:
            dave.post(f"/api/v1/experiments/{eid}/archive", {})
        assert e.value.status == 403
        carol.post(f"/api/v1/experiments/{eid}/archive", {})
        admin.post(f"/api/v1/experiments/{eid}/unarchive", {})
    finally:
        srv.stop()
        srv.master.close()


def test_cli_login_workspace_project(rbac_master, tmp_path, monkeypatch, capsys):
    url, _ = rbac_master
    monkeypatch.setenv("DET_AUTH_FILE", str(tmp_path / "auth.json"))
    import importlib

    import determined_amd.cli._iam as cli_iam

    importlib.reload(cli_iam)
    from determined_amd.cli import main

    assert main(["-m", url, "user", "login", "admin", "--password", ""]) == 0
    assert oct(os.stat(tmp_path / "auth.json").st_mode & 0o777) == "0o600"
    assert main(["-m", url, "user", "whoami"]) == 0
    assert "admin" in capsys.readouterr().out
    assert main(["-m", url, "workspace", "create", "cli-ws"]) == 0
    assert main(["-m", url, "project", "create", "cli-ws", "p1", "--description", "d"]) == 0
    assert main(["-m", url, "--json", "project", "list", "cli-ws"]) == 0
    assert '"p1"' in capsys.readouterr().out
    assert main(["-m", url, "user", "create", "erin", "--password", "z"]) == 0
    assert main(["-m", url, "rbac", "assign-role", "Editor", "--username-to-assign", "erin",
                 "--workspace-name", "cli-ws"]) == 0
    assert main(["-m", url, "--json", "rbac", "list-users-roles", "erin"]) == 0
    assert '"Editor"' in capsys.readouterr().out
    assert main(["-m", url, "user", "logout"]) == 0
    assert main(["-m", url, "user", "whoami"]) == 1


def test_sdk_users_workspaces_projects(rbac_master):
    """The SDK's user / workspace / project objects (reference ``experimental/client.py`` +
    ``common/experimental/{user,workspace,project}.py``) over the RBAC master."""
    from determined_amd.experimental import client

    url, _ = rbac_master
    client.login(url, user="admin", password="")
    try:
        assert client.whoami().username == "admin" and client.get_session_username() == "admin"
        u = client.create_user("sdk-user", password="pw1", display_name="SDK")
        assert client.get_user_by_name("sdk-user").user_id == u.user_id
        assert client.get_user_by_id(u.user_id).display_name == "SDK"
        u.change_display_name("Renamed")
        u.rename("sdk-user2")
        u.deactivate()
        assert not client.get_user_by_id(u.user_id).active
        assert "sdk-user2" in {x.username for x in client.list_users(active=False)}
        u.activate()
        u.change_password("pw2")
        with pytest.raises(APIException):
            _login(url, "sdk-user2", "pw1")
        _login(url, "sdk-user2", "pw2")
        w = client.create_workspace("sdk-ws")
        assert client.get_workspace("sdk-ws").id == w.id
        assert "sdk-ws" in {x.name for x in client.list_workspaces()}
        p = w.create_project("sdk-proj", "first")
        assert w.get_project("sdk-proj").id == p.id and p.description == "first"
        p.set_description("second")
        p.reload()
        assert p.description == "second" and p.list_experiments() == []
        p.archive()
        assert p.archived
        p.unarchive()
        w.delete_project("sdk-proj")
        assert w.list_projects() == []
        client.delete_workspace("sdk-ws")
        assert "sdk-ws" not in {x.name for x in client.list_workspaces()}
    finally:
        client.logout()
