"""``det user|workspace|project|rbac`` and ``det experiment move`` (reference:
``harness/determined/cli/{user,workspace,project,rbac}.py``).  ``det user login`` stores the
session token per master URL in ``~/.det_amd/auth.json`` (mode 0600); every later command picks
it up (``DET_MASTER_TOKEN`` overrides)."""

import argparse
import getpass
import json
import os
import pathlib
from typing import Any, Dict, Optional

AUTH_FILE = pathlib.Path(os.environ.get("DET_AUTH_FILE", str(pathlib.Path.home() / ".det_amd" / "auth.json")))


def _load_tokens() -> Dict[str, Any]:
    try:
        return json.loads(AUTH_FILE.read_text())
    except (OSError, ValueError):
        return {}


def stored_token(master: str) -> Optional[str]:
    ent = _load_tokens().get(master.rstrip("/"))
    return ent.get("token") if isinstance(ent, dict) else None


def _store_token(master: str, user: str, token: Optional[str]) -> None:
    d = _load_tokens()
    if token is None:
        d.pop(master.rstrip("/"), None)
    else:
        d[master.rstrip("/")] = {"username": user, "token": token}
    AUTH_FILE.parent.mkdir(parents=True, exist_ok=True)
    AUTH_FILE.write_text(json.dumps(d))
    os.chmod(AUTH_FILE, 0o600)


def _password(a: argparse.Namespace, prompt: str = "Password: ") -> str:
    if getattr(a, "password", None) is not None:
        return a.password
    env = os.environ.get("DET_PASS")
    return env if env is not None else getpass.getpass(prompt)


def register(sub: Any, session: Any, show: Any) -> None:
    """Add the IAM command groups to the ``det`` parser."""

    # ---------------------------------------------------------------- user
    def login(a):
        from determined_amd.common.api import Session

        out = Session(a.master).post("/api/v1/auth/login", {"username": a.username, "password": _password(a)})
        _store_token(a.master, a.username, out["token"])
        print(f"logged in as {a.username}")

    def logout(a):
        try:
            session(a).post("/api/v1/auth/logout", {})
        finally:
            _store_token(a.master, "", None)

    def whoami(a):
        u = session(a).get("/api/v1/me")["user"]
        print(f"You are logged in as user '{u['username']}'" + (" (admin)" if u["admin"] else ""))

    def user_list(a):
        show(session(a).get("/api/v1/users")["users"], ["id", "username", "display_name", "admin", "active"], a)

    def user_create(a):
        u = session(a).post("/api/v1/users", {"username": a.username, "admin": a.admin,
                                              "password": a.password or ""})["user"]
        print(f"created user {u['username']} (id {u['id']})")

    def user_patch(body):
        def fn(a):
            session(a).patch(f"/api/v1/users/{a.username}", body)
        return fn

    def user_password(a):
        target = a.target or session(a).get("/api/v1/me")["user"]["username"]
        session(a).post(f"/api/v1/users/{target}/password", {"password": _password(a, "New password: ")})
        print(f"password of {target} changed")

    u = sub.add_parser("user", aliases=["u"]).add_subparsers(dest="verb", required=True)
    p = u.add_parser("login")
    p.add_argument("username", nargs="?", default="determined")
    p.add_argument("--password", default=None)
    p.set_defaults(fn=login)
    u.add_parser("logout").set_defaults(fn=logout)
    u.add_parser("whoami").set_defaults(fn=whoami)
    u.add_parser("list").set_defaults(fn=user_list)
    p = u.add_parser("create")
    p.add_argument("username")
    p.add_argument("--admin", action="store_true")
    p.add_argument("--password", default=None)
    p.set_defaults(fn=user_create)
    for verb, body in (("activate", {"active": True}), ("deactivate", {"active": False}),
                       ("make-admin", {"admin": True}), ("remove-admin", {"admin": False})):
        p = u.add_parser(verb)
        p.add_argument("username")
        p.set_defaults(fn=user_patch(body))
    p = u.add_parser("change-password")
    p.add_argument("target", nargs="?", default=None)
    p.add_argument("--password", default=None)
    p.set_defaults(fn=user_password)

    # ---------------------------------------------------------------- workspace
    def ws_list(a):
        show(session(a).get("/api/v1/workspaces")["workspaces"], ["id", "name", "num_projects", "archived"], a)

    def ws_create(a):
        w = session(a).post("/api/v1/workspaces", {"name": a.name})["workspace"]
        print(f"created workspace {w['name']} (id {w['id']})")

    def ws_describe(a):
        s = session(a)
        w = s.get(f"/api/v1/workspaces/{a.name}")["workspace"]
        print(json.dumps(w, indent=2, default=str))
        show(s.get(f"/api/v1/workspaces/{a.name}/projects")["projects"],
             ["id", "name", "description", "num_experiments", "archived"], a)

    def ws_action(verb):
        def fn(a):
            s = session(a)
            if verb == "delete":
                s.delete(f"/api/v1/workspaces/{a.name}")
            else:
                s.post(f"/api/v1/workspaces/{a.name}/{verb}", {})
        return fn

    w = sub.add_parser("workspace", aliases=["w"]).add_subparsers(dest="verb", required=True)
    w.add_parser("list").set_defaults(fn=ws_list)
    for verb, fn in (("create", ws_create), ("describe", ws_describe), ("archive", ws_action("archive")),
                     ("unarchive", ws_action("unarchive")), ("delete", ws_action("delete"))):
        p = w.add_parser(verb)
        p.add_argument("name")
        p.set_defaults(fn=fn)

    # ---------------------------------------------------------------- project
    def proj_id(s, ws: str, name: str) -> int:
        for p in s.get(f"/api/v1/workspaces/{ws}/projects")["projects"]:
            if p["name"] == name or str(p["id"]) == name:
                return int(p["id"])
        raise SystemExit(f"project {ws}/{name} not found")

    def proj_list(a):
        show(session(a).get(f"/api/v1/workspaces/{a.workspace}/projects")["projects"],
             ["id", "name", "description", "num_experiments", "archived"], a)

    def proj_create(a):
        p = session(a).post(f"/api/v1/workspaces/{a.workspace}/projects",
                            {"name": a.name, "description": a.description})["project"]
        print(f"created project {a.workspace}/{p['name']} (id {p['id']})")

    def proj_describe(a):
        s = session(a)
        pid = proj_id(s, a.workspace, a.name)
        show(s.get(f"/api/v1/projects/{pid}/experiments")["experiments"], ["id", "name", "state", "owner"], a)

    def proj_action(verb):
        def fn(a):
            s = session(a)
            pid = proj_id(s, a.workspace, a.name)
            s.delete(f"/api/v1/projects/{pid}") if verb == "delete" else s.post(f"/api/v1/projects/{pid}/{verb}", {})
        return fn

    pr = sub.add_parser("project", aliases=["p"]).add_subparsers(dest="verb", required=True)
    p = pr.add_parser("list")
    p.add_argument("workspace")
    p.set_defaults(fn=proj_list)
    for verb, fn in (("create", proj_create), ("describe", proj_describe), ("archive", proj_action("archive")),
                     ("unarchive", proj_action("unarchive")), ("delete", proj_action("delete"))):
        p = pr.add_parser(verb)
        p.add_argument("workspace")
        p.add_argument("name")
        if verb == "create":
            p.add_argument("--description", default="")
        p.set_defaults(fn=fn)

    # ---------------------------------------------------------------- rbac
    def roles(a):
        show(session(a).get("/api/v1/rbac/roles")["roles"], ["name", "rank", "permissions"], a)

    def assignments(a):
        q = f"?user={a.username}" if a.username else ""
        show(session(a).get(f"/api/v1/rbac/assignments{q}")["assignments"], ["username", "role", "workspace"], a)

    def assign(remove):
        def fn(a):
            if bool(a.username) == bool(a.group_name):
                raise SystemExit("give exactly one of --username-to-assign / --group-name-to-assign")
            if a.group_name:
                session(a).post("/api/v1/rbac/unassign-group" if remove else "/api/v1/rbac/assign-group",
                                {"group": a.group_name, "role": a.role, "workspace": a.workspace_name})
                return
            session(a).post("/api/v1/rbac/unassign" if remove else "/api/v1/rbac/assign",
                            {"user": a.username, "role": a.role, "workspace": a.workspace_name})
        return fn

    rb = sub.add_parser("rbac").add_subparsers(dest="verb", required=True)
    rb.add_parser("list-roles").set_defaults(fn=roles)
    p = rb.add_parser("list-users-roles")
    p.add_argument("username", nargs="?", default=None)
    p.set_defaults(fn=assignments)
    for verb, remove in (("assign-role", False), ("unassign-role", True)):
        p = rb.add_parser(verb)
        p.add_argument("role")
        p.add_argument("--username-to-assign", "--username", dest="username", default=None)
        p.add_argument("--group-name-to-assign", "--group-name", dest="group_name", default=None)
        p.add_argument("--workspace-name", default=None)
        p.set_defaults(fn=assign(remove))


def register_experiment_move(exp_sub: Any, session: Any) -> None:
    def move(a):
        s = session(a)
        pid = None
        for p in s.get(f"/api/v1/workspaces/{a.workspace}/projects")["projects"]:
            if p["name"] == a.project:
                pid = p["id"]
        if pid is None:
            raise SystemExit(f"project {a.workspace}/{a.project} not found")
        s.post(f"/api/v1/experiments/{a.id}/move", {"destination_project_id": pid})
        print(f"moved experiment {a.id} to {a.workspace}/{a.project}")

    p = exp_sub.add_parser("move")
    p.add_argument("id", type=int)
    p.add_argument("workspace")
    p.add_argument("project")
    p.set_defaults(fn=move)
