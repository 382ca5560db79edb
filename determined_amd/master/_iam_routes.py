"""REST routes for users, sessions, workspaces, projects and RBAC (reference:
``master/internal/api_user.go``, ``api_workspace.go``, ``api_project.go``, ``rbac/api_rbac.go``).
Registered by ``_server.build_routes``; all business rules live in ``_iam.IAM``."""

from typing import Any, Callable

from determined_amd.master._iam import AuthError, _public_user


def add_iam_routes(route: Callable[[str, str], Callable], m: Any) -> None:
    iam = m.iam

    # ---------------------------------------------------------------- sessions
    @route("POST", "/api/v1/auth/logout")
    def logout(q, b):
        iam.logout()
        return {}

    # ---------------------------------------------------------------- users
    @route("GET", "/api/v1/users")
    def list_users(q, b):
        return {"users": iam.list_users()}

    @route("POST", "/api/v1/users")
    def create_user(q, b):
        u = b.get("user", b)
        return {"user": iam.create_user(u["username"], b.get("password", u.get("password", "")),
                                        bool(u.get("admin", False)), bool(u.get("active", True)),
                                        u.get("display_name", ""))}

    @route("GET", r"/api/v1/users/([^/]+)")
    def get_user(q, b, ref):
        return {"user": _public_user(iam.get_user(ref))}

    @route("PATCH", r"/api/v1/users/([^/]+)")
    def patch_user(q, b, ref):
        return {"user": iam.patch_user(ref, b)}

    @route("POST", r"/api/v1/users/([^/]+)/password")
    def set_password(q, b, ref):
        return {"user": iam.patch_user(ref, {"password": b.get("password", "")})}

    # ---------------------------------------------------------------- workspaces
    @route("GET", "/api/v1/workspaces")
    def list_ws(q, b):
        return {"workspaces": iam.list_workspaces()}

    @route("POST", "/api/v1/workspaces")
    def create_ws(q, b):
        return {"workspace": iam.create_workspace(b["name"])}

    @route("GET", r"/api/v1/workspaces/([^/]+)")
    def get_ws(q, b, ref):
        w = iam.workspace(ref)
        iam.require("view", w["id"])
        return {"workspace": w}

    @route("PATCH", r"/api/v1/workspaces/([^/]+)")
    def patch_ws(q, b, ref):
        return {"workspace": iam.patch_workspace(ref, b)}

    @route("POST", r"/api/v1/workspaces/([^/]+)/archive")
    def archive_ws(q, b, ref):
        return {"workspace": iam.patch_workspace(ref, {"archived": True})}

    @route("POST", r"/api/v1/workspaces/([^/]+)/unarchive")
    def unarchive_ws(q, b, ref):
        return {"workspace": iam.patch_workspace(ref, {"archived": False})}

    @route("DELETE", r"/api/v1/workspaces/([^/]+)")
    def delete_ws(q, b, ref):
        iam.delete_workspace(ref)
        return {}

    @route("GET", r"/api/v1/workspaces/([^/]+)/projects")
    def ws_projects(q, b, ref):
        return {"projects": iam.list_projects(ref)}

    @route("POST", r"/api/v1/workspaces/([^/]+)/projects")
    def create_project(q, b, ref):
        return {"project": iam.create_project(ref, b["name"], b.get("description", ""))}

    # ---------------------------------------------------------------- projects
    @route("GET", r"/api/v1/projects/(\d+)")
    def get_project(q, b, pid):
        p = iam.project(pid)
        iam.require("view", p["workspace_id"])
        return {"project": p}

    @route("PATCH", r"/api/v1/projects/(\d+)")
    def patch_project(q, b, pid):
        return {"project": iam.patch_project(pid, b)}

    @route("POST", r"/api/v1/projects/(\d+)/archive")
    def archive_project(q, b, pid):
        return {"project": iam.patch_project(pid, {"archived": True})}

    @route("POST", r"/api/v1/projects/(\d+)/unarchive")
    def unarchive_project(q, b, pid):
        return {"project": iam.patch_project(pid, {"archived": False})}

    @route("DELETE", r"/api/v1/projects/(\d+)")
    def delete_project(q, b, pid):
        iam.delete_project(pid)
        return {}

    @route("GET", r"/api/v1/projects/(\d+)/experiments")
    def project_exps(q, b, pid):
        p = iam.project(pid)
        w = iam.workspace(p["workspace_id"])
        iam.require("view", w["id"])
        rows = m.db.all("SELECT id, name, state, owner FROM experiments WHERE workspace=? AND project=? "
                        "AND state!='DELETED' ORDER BY id", [w["name"], p["name"]])
        return {"experiments": rows}

    @route("POST", r"/api/v1/experiments/(\d+)/move")
    def move_exp(q, b, eid):
        row = m.db.one("SELECT id, owner, workspace FROM experiments WHERE id=?", [int(eid)])
        if row is None:
            raise AuthError(404, f"experiment {eid} not found")
        sc = iam.experiment_scope(row)
        iam.require("edit", sc["workspace_id"], sc["owner_id"])
        p = iam.project(b["destination_project_id"])
        w = iam.workspace(p["workspace_id"])
        iam.require("edit", w["id"])
        if p["archived"] or w["archived"]:
            raise AuthError(400, "destination project is archived")
        m.db.update("experiments", "id", int(eid), project=p["name"], workspace=w["name"])
        return {}

    # ---------------------------------------------------------------- user groups
    @route("GET", "/api/v1/groups")
    def list_groups(q, b):
        return {"groups": iam.list_groups(q.get("user"))}

    @route("POST", "/api/v1/groups")
    def create_group(q, b):
        return {"group": iam.create_group(b["name"], b.get("add_users"))}

    @route("GET", r"/api/v1/groups/([^/]+)")
    def get_group(q, b, ref):
        return {"group": iam.group(ref)}

    @route("PATCH", r"/api/v1/groups/([^/]+)")
    def patch_group(q, b, ref):
        g = iam.group(ref)
        if b.get("name"):
            g = iam.rename_group(ref, b["name"])
        if b.get("add_users"):
            g = iam.set_members(g["id"], b["add_users"], add=True)
        if b.get("remove_users"):
            g = iam.set_members(g["id"], b["remove_users"], add=False)
        return {"group": g}

    @route("DELETE", r"/api/v1/groups/([^/]+)")
    def delete_group(q, b, ref):
        iam.delete_group(ref)
        return {}

    # ---------------------------------------------------------------- RBAC
    @route("GET", "/api/v1/rbac/my-permissions")
    def my_perms(q, b):
        return iam.my_permissions()

    @route("GET", "/api/v1/rbac/group-assignments")
    def group_assignments(q, b):
        return {"assignments": iam.group_assignments()}

    @route("POST", "/api/v1/rbac/assign-group")
    def assign_group(q, b):
        iam.assign_group(b["group"], b["role"], b.get("workspace"))
        return {}

    @route("POST", "/api/v1/rbac/unassign-group")
    def unassign_group(q, b):
        iam.assign_group(b["group"], b["role"], b.get("workspace"), remove=True)
        return {}

    @route("GET", "/api/v1/rbac/roles")
    def roles(q, b):
        return {"roles": iam.list_roles()}

    @route("GET", "/api/v1/rbac/assignments")
    def assignments(q, b):
        return {"assignments": iam.assignments(q.get("user"))}

    @route("POST", "/api/v1/rbac/assign")
    def assign(q, b):
        iam.assign(str(b["user"]), b["role"], b.get("workspace"))
        return {}

    @route("POST", "/api/v1/rbac/unassign")
    def unassign(q, b):
        iam.assign(str(b["user"]), b["role"], b.get("workspace"), remove=True)
        return {}
