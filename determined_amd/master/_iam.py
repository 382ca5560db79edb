"""Users, sessions, workspaces, projects and role-based access control for the master
(reference: ``master/internal/user``, ``master/internal/workspace``, ``master/internal/project``,
``master/internal/rbac`` with ``authz_basic_impl.go`` / ``authz_rbac.go`` /
``authz_permissive.go``).

Three authorization modes, chosen when the master starts:

* ``none``   -- no credentials needed; every request acts as the built-in ``determined`` user
  with full rights (single-user node; what ``det deploy local`` uses by default);
* ``basic``  -- a session token (``POST /api/v1/auth/login``) or the cluster token is required;
  admins may do anything, other users may view everything and modify what they own;
* ``rbac``   -- as ``basic`` for authentication, but permissions come from role assignments,
  global or scoped to a workspace: ``ClusterAdmin`` > ``WorkspaceAdmin`` > ``Editor`` >
  ``Viewer``, plus ``WorkspaceCreator``.

The cluster token given to agents and tasks authenticates as the internal ``determined``
admin.  Passwords are stored as salted PBKDF2-SHA256 hashes; session tokens are random and
expire (7 days by default).
"""

import hashlib
import hmac
import secrets
import threading
import time
from typing import Any, Dict, List, Optional

SCHEMA = """
CREATE TABLE IF NOT EXISTS users (
  id INTEGER PRIMARY KEY AUTOINCREMENT, username TEXT UNIQUE, display_name TEXT DEFAULT '',
  password_hash TEXT DEFAULT '', admin INTEGER DEFAULT 0, active INTEGER DEFAULT 1, created REAL);
CREATE TABLE IF NOT EXISTS user_sessions (token TEXT PRIMARY KEY, user_id INTEGER, expiry REAL);
CREATE TABLE IF NOT EXISTS workspaces (
  id INTEGER PRIMARY KEY AUTOINCREMENT, name TEXT UNIQUE, archived INTEGER DEFAULT 0, user_id INTEGER,
  created REAL, checkpoint_storage TEXT);
CREATE TABLE IF NOT EXISTS projects (
  id INTEGER PRIMARY KEY AUTOINCREMENT, name TEXT, workspace_id INTEGER, description TEXT DEFAULT '',
  archived INTEGER DEFAULT 0, user_id INTEGER, created REAL, UNIQUE(workspace_id, name));
CREATE TABLE IF NOT EXISTS role_assignments (
  id INTEGER PRIMARY KEY AUTOINCREMENT, user_id INTEGER, role TEXT, workspace_id INTEGER,
  UNIQUE(user_id, role, workspace_id));
CREATE TABLE IF NOT EXISTS user_groups (id INTEGER PRIMARY KEY AUTOINCREMENT, name TEXT UNIQUE, created REAL);
CREATE TABLE IF NOT EXISTS group_members (group_id INTEGER, user_id INTEGER, PRIMARY KEY (group_id, user_id));
CREATE TABLE IF NOT EXISTS group_role_assignments (
  id INTEGER PRIMARY KEY AUTOINCREMENT, group_id INTEGER, role TEXT, workspace_id INTEGER,
  UNIQUE(group_id, role, workspace_id));
"""
# the user's identity on the agents (reference ``det user link-with-agent-user``): tasks the user
# owns run with this uid/gid where the agent may switch users (it runs as root)
AGENT_USER_COLS = (("agent_uid", "INTEGER"), ("agent_gid", "INTEGER"), ("agent_user", "TEXT"), ("agent_group", "TEXT"))

# permission -> minimum role rank (scoped roles are checked against the object's workspace)
ROLES = {"Viewer": 1, "Editor": 2, "WorkspaceAdmin": 3, "ClusterAdmin": 4, "WorkspaceCreator": 0}
PERMS = {
    "view": 1,                 # read experiments/trials/checkpoints/models/projects
    "edit": 2,                 # create/pause/kill/archive experiments, register models
    "admin_workspace": 3,      # rename/archive/delete workspace & projects, assign roles in it
    "admin_cluster": 4,        # users, agents, global role assignments, master config
}
SESSION_TTL_S = 7 * 24 * 3600
DEFAULT_WORKSPACE = "Uncategorized"
DEFAULT_PROJECT = "Uncategorized"


class AuthError(Exception):
    def __init__(self, status: int, message: str) -> None:
        super().__init__(message)
        self.status = status
        self.message = message


def hash_password(password: str, salt: Optional[str] = None) -> str:
    salt = salt or secrets.token_hex(8)
    dk = hashlib.pbkdf2_hmac("sha256", password.encode(), salt.encode(), 20000)
    return f"pbkdf2${salt}${dk.hex()}"


def check_password(password: str, stored: str) -> bool:
    if not stored:
        return password == ""
    try:
        _, salt, _ = stored.split("$")
    except ValueError:
        return False
    return hmac.compare_digest(hash_password(password, salt), stored)


def _public_user(u: Dict[str, Any]) -> Dict[str, Any]:
    out = {"id": u["id"], "username": u["username"], "display_name": u.get("display_name") or "",
           "admin": bool(u["admin"]), "active": bool(u["active"])}
    agent = {k: u.get(k) for k, _ in AGENT_USER_COLS if u.get(k) is not None}
    if agent:
        out["agent_user_group"] = agent
    return out


class IAM:
    def __init__(self, db: Any, mode: str = "none", cluster_token: Optional[str] = None) -> None:
        if mode not in ("none", "basic", "rbac"):
            raise ValueError(f"auth mode must be none/basic/rbac, got {mode!r}")
        self.db = db
        self.mode = mode
        self.cluster_token = cluster_token
        self._local = threading.local()
        db.conn.executescript(SCHEMA)
        have = {r[1] for r in db.conn.execute("PRAGMA table_info(users)").fetchall()}
        for col, typ in AGENT_USER_COLS:
            if col not in have:
                db.conn.execute(f"ALTER TABLE users ADD COLUMN {col} {typ}")
        self._bootstrap()

    # ------------------------------------------------------------------ bootstrap
    def _bootstrap(self) -> None:
        for name, admin in (("admin", 1), ("determined", 1 if self.mode == "none" else 0)):
            if self.db.one("SELECT id FROM users WHERE username=?", [name]) is None:
                self.db.insert("users", username=name, admin=admin, active=1, created=time.time())
        if self.db.one("SELECT id FROM workspaces WHERE name=?", [DEFAULT_WORKSPACE]) is None:
            wid = self.db.insert("workspaces", name=DEFAULT_WORKSPACE, user_id=1, created=time.time())
            self.db.insert("projects", name=DEFAULT_PROJECT, workspace_id=wid, user_id=1, created=time.time())

    # ------------------------------------------------------------------ request identity
    def authenticate(self, authorization: Optional[str]) -> Dict[str, Any]:
        """Resolve the ``Authorization`` header to a user row (raises AuthError 401)."""
        tok = authorization[7:] if authorization and authorization.startswith("Bearer ") else None
        self._local.token = tok
        # a master started with a cluster token keeps requiring a credential even in mode none
        required = self.mode != "none" or self.cluster_token is not None
        if tok and self.cluster_token and hmac.compare_digest(tok, self.cluster_token):
            u = dict(self._user_by_name("determined"))
            u["admin"] = 1  # the cluster identity (agents, tasks) is trusted
            return u
        if tok:
            row = self.db.one("SELECT user_id, expiry FROM user_sessions WHERE token=?", [tok])
            if row is not None and row["expiry"] > time.time():
                u = self.db.one("SELECT * FROM users WHERE id=?", [row["user_id"]])
                if u is not None and u["active"]:
                    return u
            if required:
                raise AuthError(401, "invalid or expired session token")
        if not required:
            return self._user_by_name("determined")
        raise AuthError(401, "authentication required")

    def set_current(self, user: Optional[Dict[str, Any]]) -> None:
        self._local.user = user

    def current(self) -> Dict[str, Any]:
        u = getattr(self._local, "user", None)
        return u if u is not None else self._user_by_name("determined")

    def _user_by_name(self, name: str) -> Dict[str, Any]:
        u = self.db.one("SELECT * FROM users WHERE username=?", [name])
        if u is None:
            raise AuthError(404, f"user {name} not found")
        return u

    # ------------------------------------------------------------------ sessions
    def login(self, username: str, password: str) -> Dict[str, Any]:
        u = self.db.one("SELECT * FROM users WHERE username=?", [username])
        if u is None or not u["active"] or not check_password(password or "", u["password_hash"] or ""):
            raise AuthError(401, "invalid credentials")
        tok = secrets.token_urlsafe(32)
        self.db.insert("user_sessions", token=tok, user_id=u["id"], expiry=time.time() + SESSION_TTL_S)
        return {"token": tok, "user": _public_user(u)}

    def logout(self) -> None:
        """End the session the current request authenticated with."""
        tok = getattr(self._local, "token", None)
        if tok:
            self.db.execute("DELETE FROM user_sessions WHERE token=?", [tok])

    # ------------------------------------------------------------------ authorization
    def _rank(self, user: Dict[str, Any], workspace_id: Optional[int]) -> int:
        if user["admin"]:
            return ROLES["ClusterAdmin"]
        rows = self._role_rows(user)
        best = 0
        for r in rows:
            if r["workspace_id"] is None or (workspace_id is not None and r["workspace_id"] == workspace_id):
                best = max(best, ROLES.get(r["role"], 0))
        return best

    def has_role(self, user: Dict[str, Any], role: str, workspace_id: Optional[int] = None) -> bool:
        if user["admin"]:
            return True
        rows = [r for r in self._role_rows(user) if r["role"] == role]
        return any(r["workspace_id"] is None or r["workspace_id"] == workspace_id for r in rows)

    def _role_rows(self, user: Dict[str, Any]) -> List[Dict[str, Any]]:
        """The user's own role assignments plus those of every group it belongs to."""
        return self.db.all("SELECT role, workspace_id FROM role_assignments WHERE user_id=? UNION ALL "
                           "SELECT g.role, g.workspace_id FROM group_role_assignments g JOIN group_members m "
                           "ON m.group_id = g.group_id WHERE m.user_id=?", [user["id"], user["id"]])

    def can(self, perm: str, workspace_id: Optional[int] = None, owner_id: Optional[int] = None,
            user: Optional[Dict[str, Any]] = None) -> bool:
        user = user or self.current()
        if self.mode == "none" or user["admin"]:
            return True
        need = PERMS[perm]
        if self.mode == "basic":
            if need <= PERMS["view"]:
                return True
            if need == PERMS["admin_cluster"]:
                return False
            if owner_id is None:  # creating something new (experiment, project) is open to all
                return need <= PERMS["edit"]
            return owner_id == user["id"]
        if owner_id is not None and owner_id == user["id"] and need <= PERMS["edit"]:
            return True
        return self._rank(user, workspace_id) >= need

    def require(self, perm: str, workspace_id: Optional[int] = None, owner_id: Optional[int] = None) -> None:
        if not self.can(perm, workspace_id, owner_id):
            u = self.current()
            raise AuthError(403, f"user {u['username']} lacks permission '{perm}'"
                            + (f" on workspace {workspace_id}" if workspace_id is not None else ""))

    # ------------------------------------------------------------------ users
    def list_users(self) -> List[Dict[str, Any]]:
        return [_public_user(u) for u in self.db.all("SELECT * FROM users ORDER BY id")]

    def get_user(self, ref: str) -> Dict[str, Any]:
        u = self.db.one("SELECT * FROM users WHERE id=?", [int(ref)]) if str(ref).isdigit() else \
            self.db.one("SELECT * FROM users WHERE username=?", [ref])
        if u is None:
            raise AuthError(404, f"user {ref} not found")
        return u

    def create_user(self, username: str, password: str = "", admin: bool = False, active: bool = True,
                    display_name: str = "") -> Dict[str, Any]:
        self.require("admin_cluster")
        if not username or self.db.one("SELECT id FROM users WHERE username=?", [username]) is not None:
            raise AuthError(409, f"user {username!r} already exists")
        uid = self.db.insert("users", username=username, admin=int(admin), active=int(active),
                             display_name=display_name, password_hash=hash_password(password) if password else "",
                             created=time.time())
        return _public_user(self.get_user(str(uid)))

    def patch_user(self, ref: str, body: Dict[str, Any]) -> Dict[str, Any]:
        u = self.get_user(ref)
        me = self.current()
        self_edit = me["id"] == u["id"]
        if not (self_edit and set(body) <= {"password", "display_name"}):
            self.require("admin_cluster")
        cols: Dict[str, Any] = {}
        if "password" in body:
            cols["password_hash"] = hash_password(body["password"]) if body["password"] else ""
            self.db.execute("DELETE FROM user_sessions WHERE user_id=?", [u["id"]])
        for k in ("display_name",):
            if k in body:
                cols[k] = body[k]
        if "username" in body and body["username"] != u["username"]:  # rename (admin only, above)
            if not body["username"] or self.db.one("SELECT id FROM users WHERE username=?", [body["username"]]):
                raise AuthError(400, f"username {body['username']!r} is empty or taken")
            cols["username"] = body["username"]
        for k in ("admin", "active"):
            if k in body:
                cols[k] = int(bool(body[k]))
        for k, _ in AGENT_USER_COLS:  # link-with-agent-user (admin only, checked above)
            if k in body:
                cols[k] = body[k]
        if cols:
            self.db.update("users", "id", u["id"], **cols)
        return _public_user(self.get_user(str(u["id"])))

    # ------------------------------------------------------------------ workspaces / projects
    def workspace(self, ref: Any) -> Dict[str, Any]:
        w = self.db.one("SELECT * FROM workspaces WHERE id=?", [int(ref)]) if str(ref).isdigit() else \
            self.db.one("SELECT * FROM workspaces WHERE name=?", [ref])
        if w is None:
            raise AuthError(404, f"workspace {ref} not found")
        return w

    def list_workspaces(self) -> List[Dict[str, Any]]:
        out = []
        for w in self.db.all("SELECT * FROM workspaces ORDER BY id"):
            n = self.db.one("SELECT COUNT(*) AS n FROM projects WHERE workspace_id=?", [w["id"]])["n"]
            if self.can("view", w["id"]):
                out.append(dict(w, num_projects=n, archived=bool(w["archived"])))
        return out

    def create_workspace(self, name: str) -> Dict[str, Any]:
        me = self.current()
        if not (self.mode == "none" or me["admin"] or self.has_role(me, "WorkspaceCreator")
                or self.mode == "basic"):
            raise AuthError(403, f"user {me['username']} may not create workspaces")
        if not name or self.db.one("SELECT id FROM workspaces WHERE name=?", [name]) is not None:
            raise AuthError(409, f"workspace {name!r} already exists")
        wid = self.db.insert("workspaces", name=name, user_id=me["id"], created=time.time())
        if self.mode == "rbac" and not me["admin"]:
            # the creator administers what they create (reference: WorkspaceCreator semantics)
            self.db.insert("role_assignments", user_id=me["id"], role="WorkspaceAdmin", workspace_id=wid)
        return self.workspace(wid)

    def patch_workspace(self, ref: Any, body: Dict[str, Any]) -> Dict[str, Any]:
        w = self.workspace(ref)
        self.require("admin_workspace", w["id"], w["user_id"])
        if w["name"] == DEFAULT_WORKSPACE and "name" in body:
            raise AuthError(400, "the default workspace cannot be renamed")
        cols = {k: body[k] for k in ("name", "archived") if k in body}
        if "archived" in cols:
            cols["archived"] = int(bool(cols["archived"]))
        if "name" in cols:
            self.db.execute("UPDATE experiments SET workspace=? WHERE workspace=?", [cols["name"], w["name"]])
        if cols:
            self.db.update("workspaces", "id", w["id"], **cols)
        return self.workspace(w["id"])

    def delete_workspace(self, ref: Any) -> None:
        w = self.workspace(ref)
        self.require("admin_workspace", w["id"], w["user_id"])
        if w["name"] == DEFAULT_WORKSPACE:
            raise AuthError(400, "the default workspace cannot be deleted")
        n = self.db.one("SELECT COUNT(*) AS n FROM experiments WHERE workspace=?", [w["name"]])["n"]
        if n:
            raise AuthError(409, f"workspace {w['name']} still holds {n} experiments")
        self.db.execute("DELETE FROM projects WHERE workspace_id=?", [w["id"]])
        self.db.execute("DELETE FROM role_assignments WHERE workspace_id=?", [w["id"]])
        self.db.execute("DELETE FROM workspaces WHERE id=?", [w["id"]])

    def project(self, ref: Any) -> Dict[str, Any]:
        p = self.db.one("SELECT * FROM projects WHERE id=?", [int(ref)])
        if p is None:
            raise AuthError(404, f"project {ref} not found")
        return p

    def project_by_name(self, workspace: str, name: str) -> Dict[str, Any]:
        w = self.workspace(workspace)
        p = self.db.one("SELECT * FROM projects WHERE workspace_id=? AND name=?", [w["id"], name])
        if p is None:
            raise AuthError(404, f"project {workspace}/{name} not found")
        return p

    def list_projects(self, workspace_ref: Any) -> List[Dict[str, Any]]:
        w = self.workspace(workspace_ref)
        self.require("view", w["id"])
        out = []
        for p in self.db.all("SELECT * FROM projects WHERE workspace_id=? ORDER BY id", [w["id"]]):
            n = self.db.one("SELECT COUNT(*) AS n FROM experiments WHERE workspace=? AND project=?",
                            [w["name"], p["name"]])["n"]
            out.append(dict(p, workspace=w["name"], num_experiments=n, archived=bool(p["archived"])))
        return out

    def create_project(self, workspace_ref: Any, name: str, description: str = "") -> Dict[str, Any]:
        w = self.workspace(workspace_ref)
        self.require("edit", w["id"])
        if w["archived"]:
            raise AuthError(400, f"workspace {w['name']} is archived")
        if not name or self.db.one("SELECT id FROM projects WHERE workspace_id=? AND name=?",
                                   [w["id"], name]) is not None:
            raise AuthError(409, f"project {name!r} already exists in {w['name']}")
        pid = self.db.insert("projects", name=name, workspace_id=w["id"], description=description,
                             user_id=self.current()["id"], created=time.time())
        return self.project(pid)

    def patch_project(self, ref: Any, body: Dict[str, Any]) -> Dict[str, Any]:
        p = self.project(ref)
        w = self.workspace(p["workspace_id"])
        self.require("admin_workspace", w["id"], p["user_id"])
        cols = {k: body[k] for k in ("name", "description", "archived") if k in body}
        if "archived" in cols:
            cols["archived"] = int(bool(cols["archived"]))
        if "name" in cols:
            self.db.execute("UPDATE experiments SET project=? WHERE workspace=? AND project=?",
                            [cols["name"], w["name"], p["name"]])
        if cols:
            self.db.update("projects", "id", p["id"], **cols)
        return self.project(p["id"])

    def delete_project(self, ref: Any) -> None:
        p = self.project(ref)
        w = self.workspace(p["workspace_id"])
        self.require("admin_workspace", w["id"], p["user_id"])
        n = self.db.one("SELECT COUNT(*) AS n FROM experiments WHERE workspace=? AND project=?",
                        [w["name"], p["name"]])["n"]
        if n:
            raise AuthError(409, f"project {p['name']} still holds {n} experiments")
        self.db.execute("DELETE FROM projects WHERE id=?", [p["id"]])

    def resolve_target(self, cfg: Dict[str, Any]) -> Dict[str, Any]:
        """Workspace/project an experiment config targets; checks edit rights and archival."""
        wname = cfg.get("workspace") or DEFAULT_WORKSPACE
        pname = cfg.get("project") or DEFAULT_PROJECT
        w = self.workspace(wname)
        p = self.db.one("SELECT * FROM projects WHERE workspace_id=? AND name=?", [w["id"], pname])
        if p is None:
            raise AuthError(404, f"project {wname}/{pname} not found")
        if w["archived"] or p["archived"]:
            raise AuthError(400, f"{wname}/{pname} is archived")
        self.require("edit", w["id"])
        return {"workspace": w, "project": p}

    def experiment_scope(self, row: Dict[str, Any]) -> Dict[str, Any]:
        w = self.db.one("SELECT id FROM workspaces WHERE name=?", [row.get("workspace") or DEFAULT_WORKSPACE])
        owner = self.db.one("SELECT id FROM users WHERE username=?", [row.get("owner") or "determined"])
        return {"workspace_id": w["id"] if w else None, "owner_id": owner["id"] if owner else None}

    # ------------------------------------------------------------------ RBAC
    def list_roles(self) -> List[Dict[str, Any]]:
        return [{"name": r, "rank": k, "permissions": [p for p, need in PERMS.items() if 0 < need <= k]}
                for r, k in ROLES.items()]

    def assign(self, user_ref: str, role: str, workspace_ref: Any = None, remove: bool = False) -> None:
        if role not in ROLES:
            raise AuthError(400, f"unknown role {role!r}; roles: {sorted(ROLES)}")
        u = self.get_user(user_ref)
        wid = None if workspace_ref in (None, "") else self.workspace(workspace_ref)["id"]
        if wid is None or role in ("ClusterAdmin", "WorkspaceCreator"):
            self.require("admin_cluster")
        else:
            self.require("admin_workspace", wid)
        if remove:
            if wid is None:
                self.db.execute("DELETE FROM role_assignments WHERE user_id=? AND role=? AND workspace_id IS NULL",
                                [u["id"], role])
            else:
                self.db.execute("DELETE FROM role_assignments WHERE user_id=? AND role=? AND workspace_id=?",
                                [u["id"], role, wid])
            return
        if wid is None:
            exists = self.db.one("SELECT id FROM role_assignments WHERE user_id=? AND role=? AND workspace_id IS NULL",
                                 [u["id"], role])
        else:
            exists = self.db.one("SELECT id FROM role_assignments WHERE user_id=? AND role=? AND workspace_id=?",
                                 [u["id"], role, wid])
        if exists is None:
            self.db.insert("role_assignments", user_id=u["id"], role=role, workspace_id=wid)

    # ------------------------------------------------------------------ user groups
    def group(self, ref: Any) -> Dict[str, Any]:
        g = self.db.one("SELECT * FROM user_groups WHERE id=?", [int(ref)]) if str(ref).isdigit() else \
            self.db.one("SELECT * FROM user_groups WHERE name=?", [ref])
        if g is None:
            raise AuthError(404, f"user group {ref} not found")
        members = self.db.all("SELECT u.id, u.username FROM group_members m JOIN users u ON u.id = m.user_id "
                              "WHERE m.group_id=? ORDER BY u.username", [g["id"]])
        return {"id": g["id"], "name": g["name"], "members": [m["username"] for m in members],
                "num_members": len(members)}

    def list_groups(self, user_ref: Optional[str] = None) -> List[Dict[str, Any]]:
        rows = self.db.all("SELECT id FROM user_groups ORDER BY name")
        out = [self.group(r["id"]) for r in rows]
        if user_ref:
            name = self.get_user(user_ref)["username"]
            out = [g for g in out if name in g["members"]]
        return out

    def create_group(self, name: str, members: Optional[List[str]] = None) -> Dict[str, Any]:
        self.require("admin_cluster")
        if not name or self.db.one("SELECT id FROM user_groups WHERE name=?", [name]) is not None:
            raise AuthError(409, f"user group {name!r} already exists")
        gid = self.db.insert("user_groups", name=name, created=time.time())
        if members:
            self.set_members(gid, members, add=True)
        return self.group(gid)

    def rename_group(self, ref: Any, name: str) -> Dict[str, Any]:
        self.require("admin_cluster")
        g = self.group(ref)
        if not name or self.db.one("SELECT id FROM user_groups WHERE name=?", [name]) is not None:
            raise AuthError(409, f"user group {name!r} already exists")
        self.db.update("user_groups", "id", g["id"], name=name)
        return self.group(g["id"])

    def delete_group(self, ref: Any) -> None:
        self.require("admin_cluster")
        g = self.group(ref)
        for t in ("group_members", "group_role_assignments"):
            self.db.execute(f"DELETE FROM {t} WHERE group_id=?", [g["id"]])
        self.db.execute("DELETE FROM user_groups WHERE id=?", [g["id"]])

    def set_members(self, ref: Any, users: List[str], add: bool) -> Dict[str, Any]:
        self.require("admin_cluster")
        g = self.group(ref)
        for u in users:
            uid = self.get_user(u)["id"]
            if add:
                self.db.execute("INSERT OR IGNORE INTO group_members (group_id, user_id) VALUES (?, ?)", [g["id"], uid])
            else:
                self.db.execute("DELETE FROM group_members WHERE group_id=? AND user_id=?", [g["id"], uid])
        return self.group(g["id"])

    def assign_group(self, group_ref: Any, role: str, workspace_ref: Any = None, remove: bool = False) -> None:
        if role not in ROLES:
            raise AuthError(400, f"unknown role {role!r}; roles: {sorted(ROLES)}")
        g = self.group(group_ref)
        wid = None if workspace_ref in (None, "") else self.workspace(workspace_ref)["id"]
        if wid is None or role in ("ClusterAdmin", "WorkspaceCreator"):
            self.require("admin_cluster")
        else:
            self.require("admin_workspace", wid)
        where = "group_id=? AND role=? AND " + ("workspace_id IS NULL" if wid is None else "workspace_id=?")
        args = [g["id"], role] + ([] if wid is None else [wid])
        if remove:
            self.db.execute(f"DELETE FROM group_role_assignments WHERE {where}", args)
        elif self.db.one(f"SELECT id FROM group_role_assignments WHERE {where}", args) is None:
            self.db.insert("group_role_assignments", group_id=g["id"], role=role, workspace_id=wid)

    def group_assignments(self) -> List[Dict[str, Any]]:
        return self.db.all("SELECT r.id, g.name AS group_name, r.role, w.name AS workspace FROM group_role_assignments r "
                           "JOIN user_groups g ON g.id = r.group_id LEFT JOIN workspaces w ON w.id = r.workspace_id "
                           "ORDER BY r.id")

    def my_permissions(self) -> Dict[str, Any]:
        """The current user's effective permissions: cluster-wide and per workspace."""
        u = self.current()
        scopes: Dict[str, List[str]] = {}
        wss = self.db.all("SELECT id, name FROM workspaces ORDER BY id")
        for scope, wid in [("cluster", None)] + [(w["name"], w["id"]) for w in wss]:
            scopes[scope] = [p for p in PERMS if self.can(p, wid, user=u)]
        return {"username": u["username"], "mode": self.mode, "permissions": scopes}

    def assignments(self, user_ref: Optional[str] = None) -> List[Dict[str, Any]]:
        sql = ("SELECT r.id, u.username, r.role, w.name AS workspace FROM role_assignments r "
               "JOIN users u ON u.id = r.user_id LEFT JOIN workspaces w ON w.id = r.workspace_id")
        if user_ref:
            u = self.get_user(user_ref)
            return self.db.all(sql + " WHERE r.user_id=? ORDER BY r.id", [u["id"]])
        return self.db.all(sql + " ORDER BY r.id")
