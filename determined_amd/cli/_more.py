"""The rest of the reference ``det`` command tree (``harness/determined/cli/{agent,checkpoint,
command,notebook,shell,tensorboard,experiment,job,master,project,rbac,resource_pool,resources,
task,template,user,user_groups,version,workspace,dev}.py`` and ``cli.py preview-search``):
verbs added to the groups :func:`determined_amd.cli.build_parser` already created, plus the
``resources``, ``user-group``, ``version``, ``dev`` and ``preview-search`` nouns."""

import argparse
import base64
import datetime
import json
import os
import random
import sys
from typing import Any, Callable, Dict, List

import yaml


def _group(sub: argparse._SubParsersAction, noun: str) -> argparse._SubParsersAction:
    """The verb sub-parsers of an existing noun."""
    p = sub.choices[noun]
    return next(a for a in p._actions if isinstance(a, argparse._SubParsersAction))


def _add(group: argparse._SubParsersAction, name: str, fn: Callable, *args: Any, aliases=()) -> argparse.ArgumentParser:
    p = group.add_parser(name, aliases=list(aliases))
    for a in args:
        if isinstance(a, tuple):
            p.add_argument(*a[0], **a[1])
        else:
            p.add_argument(a)
    p.set_defaults(fn=fn)
    return p


def _yaml_file(path: str) -> Dict[str, Any]:
    with open(path) as f:
        return yaml.safe_load(f) or {}


def register(sub: argparse._SubParsersAction, session: Callable, show: Callable, follow_logs: Callable) -> None:
    # ---------------------------------------------------------------- agent
    def agent_toggle(enable: bool):
        def fn(a):
            session(a).post(f"/api/v1/agents/{a.agent_id}/{'enable' if enable else 'disable'}", {})
            print(f"agent {a.agent_id} {'enabled' if enable else 'disabled'}")
        return fn

    ag = _group(sub, "agent")
    _add(ag, "enable", agent_toggle(True), "agent_id")
    _add(ag, "disable", agent_toggle(False), "agent_id")

    def slot_toggle(enable: bool):  # reference cli/agent.py patch_slot
        def fn(a):
            verb = "enable" if enable else "disable"
            session(a).post(f"/api/v1/agents/{a.agent_id}/slots/{a.slot_id}/{verb}", {})
            print(f"{verb}d slot {a.slot_id} of agent {a.agent_id}")
        return fn

    sl = _group(sub, "slot")
    _add(sl, "enable", slot_toggle(True), "agent_id", (("slot_id",), {"type": int}))
    _add(sl, "disable", slot_toggle(False), "agent_id", (("slot_id",), {"type": int}))

    # ---------------------------------------------------------------- checkpoint rm / experiment aliases
    ck = _group(sub, "checkpoint")
    _add(ck, "rm", ck.choices["delete"]._defaults["fn"], (("uuids",), {"nargs": "+"}))
    ex = _group(sub, "experiment")
    for alias, verb in (("lt", "list-trials"), ("lc", "list-checkpoints"), ("unpause", "activate")):
        src = ex.choices[verb]
        p = ex.add_parser(alias)
        for act in src._actions:
            if act.dest == "help":
                continue
            p._add_action(act)
        p.set_defaults(**src._defaults)

    # ---------------------------------------------------------------- NTSC + commands: config / set priority / logs
    for noun in ("command", "notebook", "shell", "tensorboard"):
        grp = _group(sub, noun)

        def task_config(a):
            t = session(a).get(f"/api/v1/tasks/{a.task_id}")["task"]
            print(yaml.safe_dump(t.get("config") or {}, sort_keys=False), end="")

        def set_priority(a):
            session(a).post("/api/v1/job-queues/update", {"updates": [{"job_id": a.task_id, "priority": a.priority}]})
            print(f"{a.task_id}: priority {a.priority}")

        _add(grp, "config", task_config, "task_id")
        st = grp.add_parser("set").add_subparsers(dest="field", required=True)
        _add(st, "priority", set_priority, "task_id", (("priority",), {"type": int}))
        if noun == "command":
            def cmd_logs(a):
                s = session(a)
                if a.follow:
                    follow_logs(s, a.task_id, lambda: s.get(f"/api/v1/tasks/{a.task_id}")["task"]["state"] in
                                ("TERMINATED", "CANCELED"))
                    return
                for ln in s.get(f"/api/v1/tasks/{a.task_id}/logs")["logs"]:
                    print(ln["log"])

            _add(grp, "logs", cmd_logs, "task_id", (("-f", "--follow"), {"action": "store_true"}))
        for verb in ("run", "start"):
            if verb in grp.choices:  # --resource-pool / --priority on task creation
                p = grp.choices[verb]
                p.add_argument("--resource-pool", default=None)
                p.add_argument("--priority", type=int, default=None)

    # ---------------------------------------------------------------- job update
    def job_update(a):
        u = {"job_id": a.job_id}
        if a.priority is not None:
            u["priority"] = a.priority
        if a.weight is not None:
            u["weight"] = a.weight
        session(a).post("/api/v1/job-queues/update", {"updates": [u]})

    _add(_group(sub, "job"), "update", job_update, "job_id", (("--priority",), {"type": int, "default": None}),
         (("--weight",), {"type": float, "default": None}))

    # ---------------------------------------------------------------- master config show / set
    def master_show(a):
        print(yaml.safe_dump(session(a).get("/api/v1/master/config")["config"], sort_keys=False), end="")

    def master_set(a):
        cfg = session(a).patch("/api/v1/master/config", {"log": {"level": a.log_level}})["config"]
        print(f"log level: {cfg['log']['level']}")

    mc = _group(sub, "master").choices["config"]
    mcs = mc.add_subparsers(dest="cfgverb")
    _add(mcs, "show", master_show)
    _add(mcs, "set", master_set, (("--log-level", "--log.level"), {"dest": "log_level", "required": True}))

    # ---------------------------------------------------------------- project / workspace extras
    def proj_id(s, ws: str, name: str) -> int:
        for p in s.get(f"/api/v1/workspaces/{ws}/projects")["projects"]:
            if p["name"] == name or str(p["id"]) == name:
                return int(p["id"])
        raise SystemExit(f"project {ws}/{name} not found")

    def proj_exps(a):
        s = session(a)
        show(s.get(f"/api/v1/projects/{proj_id(s, a.workspace, a.name)}/experiments")["experiments"],
             ["id", "name", "state", "owner"], a)

    def proj_edit(a):
        s = session(a)
        body = {k: v for k, v in (("name", a.new_name), ("description", a.description)) if v is not None}
        p = s.patch(f"/api/v1/projects/{proj_id(s, a.workspace, a.name)}", body)["project"]
        print(f"project {a.workspace}/{p['name']} updated")

    pr = _group(sub, "project")
    _add(pr, "list-experiments", proj_exps, "workspace", "name")
    _add(pr, "edit", proj_edit, "workspace", "name", (("--name",), {"dest": "new_name", "default": None}),
         (("--description",), {"default": None}))

    def ws_projects(a):
        show(session(a).get(f"/api/v1/workspaces/{a.name}/projects")["projects"],
             ["id", "name", "description", "num_experiments", "archived"], a)

    def ws_pools(a):
        for p in session(a).get(f"/api/v1/workspaces/{a.name}/available-resource-pools")["resource_pools"]:
            print(p)

    def ws_edit(a):
        w = session(a).patch(f"/api/v1/workspaces/{a.name}", {"name": a.new_name})["workspace"]
        print(f"workspace {a.name} renamed to {w['name']}")

    ws = _group(sub, "workspace")
    _add(ws, "list-projects", ws_projects, "name")
    _add(ws, "list-pools", ws_pools, "name")
    _add(ws, "edit", ws_edit, "name", (("--name",), {"dest": "new_name", "required": True}))

    # ---------------------------------------------------------------- rbac extras
    def my_perms(a):
        r = session(a).get("/api/v1/rbac/my-permissions")
        if getattr(a, "json", False):
            print(json.dumps(r, indent=2))
            return
        print(f"user {r['username']} (auth mode {r['mode']})")
        for scope, perms in r["permissions"].items():
            print(f"  {scope:24s} {', '.join(perms) or '-'}")

    def describe_role(a):
        roles = {r["name"]: r for r in session(a).get("/api/v1/rbac/roles")["roles"]}
        if a.role not in roles:
            raise SystemExit(f"unknown role {a.role!r}; roles: {sorted(roles)}")
        print(json.dumps(roles[a.role], indent=2))

    def group_roles(a):
        show(session(a).get("/api/v1/rbac/group-assignments")["assignments"], ["group_name", "role", "workspace"], a)

    rb = _group(sub, "rbac")
    _add(rb, "my-permissions", my_perms)
    _add(rb, "describe-role", describe_role, "role")
    _add(rb, "list-groups-roles", group_roles)

    # ---------------------------------------------------------------- resource-pool bindings
    def bind(method: str):
        def fn(a):
            r = session(a).request(method, f"/api/v1/resource-pools/{a.pool}/workspace-bindings",
                                   body={"workspace_names": a.workspace_names})
            print(f"{a.pool}: bound to {', '.join(r['workspaces']) or 'no workspace (open to all)'}")
        return fn

    def bind_list(a):
        r = session(a).get(f"/api/v1/resource-pools/{a.pool}/workspace-bindings")
        for w in r["workspaces"]:
            print(w)

    rp = _group(sub, "resource-pool")
    bd = rp.add_parser("bindings").add_subparsers(dest="bverb", required=True)
    for verb, method in (("add", "POST"), ("remove", "DELETE"), ("replace", "PUT")):
        _add(bd, verb, bind(method), "pool", (("workspace_names",), {"nargs": "+"}))
    _add(bd, "list-workspaces", bind_list, "pool")

    # ---------------------------------------------------------------- resources (allocation accounting)
    def res_raw(a):
        rows = session(a).get("/api/v1/resources/allocation/raw", params={"timestamp_after": a.timestamp_after,
                                                                           "timestamp_before": a.timestamp_before})
        rows = rows["allocations"]
        if a.json:
            print(json.dumps(rows, indent=2, default=str))
            return
        cols = ["alloc_id", "kind", "experiment_id", "owner", "resource_pool", "slots", "start_time", "end_time",
                "seconds"]
        print(",".join(cols))
        for r in rows:
            print(",".join("" if r.get(c) is None else str(r.get(c)) for c in cols))

    def res_agg(a):
        r = session(a).get("/api/v1/resources/allocation/aggregated",
                           params={"start_date": a.start_date, "end_date": a.end_date,
                                   "period": "MONTHLY" if a.monthly else "DAILY"})["resource_entries"]
        if a.json:
            print(json.dumps(r, indent=2))
            return
        print("period_start,slot_hours")
        for e in r:
            print(f"{e['period_start']},{e['seconds'] / 3600:.4f}")

    res = sub.add_parser("resources", aliases=["res"]).add_subparsers(dest="verb", required=True)
    _add(res, "raw", res_raw, "timestamp_after", "timestamp_before", (("--json",), {"action": "store_true"}))
    _add(res, "aggregated", res_agg, "start_date", "end_date", (("--monthly",), {"action": "store_true"}),
         (("--json",), {"action": "store_true"}), aliases=["agg"])

    # ---------------------------------------------------------------- task extras
    def task_cleanup(a):
        print(f"removed {session(a).post('/api/v1/tasks/cleanup-logs', {})['removed']} log lines")

    def task_create(a):
        cfg = _yaml_file(a.config_file)
        ep = cfg.get("entrypoint")
        if not ep:
            raise SystemExit("the task config needs an entrypoint")
        argv = ep if isinstance(ep, list) else ["bash", "-c", str(ep)]
        body = {"command": argv, "slots": int((cfg.get("resources") or {}).get("slots", 0)),
                "resource_pool": (cfg.get("resources") or {}).get("resource_pool"),
                "env": dict(kv.split("=", 1) for kv in (cfg.get("environment") or {}).get(
                    "environment_variables", []) if "=" in kv)}
        if a.context:
            from determined_amd.cli import tar_model_dir

            body["workdir_b64"] = base64.b64encode(tar_model_dir(a.context)).decode()
        print(f"Created task {session(a).post('/api/v1/commands', body)['task_id']}")

    def task_fork(a):
        s = session(a)
        t = s.get(f"/api/v1/tasks/{a.task_id}")["task"]
        cfg = t.get("config") or {}
        r = s.post("/api/v1/commands", {"command": cfg.get("cmd"), "slots": int(cfg.get("slots", 0)),
                                        "resource_pool": cfg.get("resource_pool"), "type": t.get("type", "COMMAND"),
                                        "priority": cfg.get("priority")})
        print(f"Forked task {a.task_id} as {r['task_id']}")

    tk = _group(sub, "task")
    _add(tk, "cleanup-logs", task_cleanup)
    _add(tk, "create", task_create, "config_file", (("context",), {"nargs": "?", "default": None}))
    _add(tk, "fork", task_fork, "task_id")

    # ---------------------------------------------------------------- template extras
    def tpl_create(a):
        s = session(a)
        if any(t["name"] == a.name for t in s.get("/api/v1/templates")["templates"]):
            raise SystemExit(f"template {a.name} already exists (use `det template set`)")
        s.request("PUT", f"/api/v1/templates/{a.name}", body={"config": _yaml_file(a.file)})
        print(f"created template {a.name}")

    def tpl_patch(a):
        s = session(a)
        cur = s.get(f"/api/v1/templates/{a.name}")["template"]["config"] or {}
        _merge(cur, _yaml_file(a.file))
        s.request("PUT", f"/api/v1/templates/{a.name}", body={"config": cur})
        print(f"updated template {a.name}")

    tp = _group(sub, "template")
    _add(tp, "create", tpl_create, "name", "file")
    sv = tp.add_parser("set-value").add_subparsers(dest="field", required=True)
    _add(sv, "config", tpl_patch, "name", "file")
    _add(tp, "config", tpl_patch, "name", "file")  # reference `det template config NAME FILE`

    def task_pause(pause: bool):
        def fn(a):
            session(a).post(f"/api/v1/tasks/{a.task_id}/{'pause' if pause else 'unpause'}", {})
            print(f"{'Paused' if pause else 'Unpaused'} task: {a.task_id}")
        return fn

    _add(tk, "pause", task_pause(True), "task_id")
    _add(tk, "unpause", task_pause(False), "task_id")

    # ---------------------------------------------------------------- user extras
    def user_rename(a):
        u = session(a).patch(f"/api/v1/users/{a.username}", {"username": a.new_username})["user"]
        print(f"renamed {a.username} to {u['username']}")

    def user_edit(a):
        body: Dict[str, Any] = {}
        if a.display_name is not None:
            body["display_name"] = a.display_name
        if a.new_username is not None:
            body["username"] = a.new_username
        if a.active is not None:
            body["active"] = a.active == "true"
        if a.admin is not None:
            body["admin"] = a.admin == "true"
        u = session(a).patch(f"/api/v1/users/{a.username}", body)["user"]
        print(f"updated user {u['username']}")

    def user_link(a):
        body = {"agent_uid": a.agent_uid, "agent_gid": a.agent_gid, "agent_user": a.agent_user,
                "agent_group": a.agent_group}
        session(a).patch(f"/api/v1/users/{a.det_username}", body)
        print(f"linked {a.det_username} to agent user {a.agent_user} ({a.agent_uid}:{a.agent_gid})")

    us = _group(sub, "user")
    _add(us, "rename", user_rename, "username", "new_username")
    _add(us, "edit", user_edit, "username", (("--display-name",), {"default": None}),
         (("--username",), {"dest": "new_username", "default": None}),
         (("--active",), {"choices": ["true", "false"], "default": None}),
         (("--admin",), {"choices": ["true", "false"], "default": None}))
    _add(us, "link-with-agent-user", user_link, "det_username", (("--agent-uid",), {"type": int, "required": True}),
         (("--agent-gid",), {"type": int, "required": True}), (("--agent-user",), {"required": True}),
         (("--agent-group",), {"required": True}))

    # ---------------------------------------------------------------- user-group
    def ug_create(a):
        g = session(a).post("/api/v1/groups", {"name": a.group_name, "add_users": a.add_user or []})["group"]
        print(f"created group {g['name']} (id {g['id']}) with {g['num_members']} member(s)")

    def ug_list(a):
        params = {"user": a.groups_user_belongs_to} if a.groups_user_belongs_to else None
        show(session(a).get("/api/v1/groups", params=params)["groups"], ["id", "name", "num_members"], a)

    def ug_describe(a):
        g = session(a).get(f"/api/v1/groups/{a.group_name}")["group"]
        print(json.dumps(g, indent=2) if getattr(a, "json", False) else
              f"group {g['name']} (id {g['id']}): {', '.join(g['members']) or 'no members'}")

    def ug_members(key: str):
        def fn(a):
            g = session(a).patch(f"/api/v1/groups/{a.group_name}", {key: a.usernames.split(",")})["group"]
            print(f"group {g['name']}: {', '.join(g['members']) or 'no members'}")
        return fn

    def ug_rename(a):
        session(a).patch(f"/api/v1/groups/{a.old_group_name}", {"name": a.new_group_name})

    def ug_delete(a):
        session(a).delete(f"/api/v1/groups/{a.group_name}")
        print(f"deleted group {a.group_name}")

    ug = sub.add_parser("user-group").add_subparsers(dest="verb", required=True)
    _add(ug, "create", ug_create, "group_name", (("--add-user",), {"action": "append"}))
    _add(ug, "list", ug_list, (("--groups-user-belongs-to",), {"default": None}), aliases=["ls"])
    _add(ug, "describe", ug_describe, "group_name")
    _add(ug, "add-user", ug_members("add_users"), "group_name", "usernames")
    _add(ug, "remove-user", ug_members("remove_users"), "group_name", "usernames")
    _add(ug, "change-name", ug_rename, "old_group_name", "new_group_name")
    _add(ug, "delete", ug_delete, "group_name")

    # ---------------------------------------------------------------- version / dev
    def version(a):
        from determined_amd import __version__

        print(f"client: {__version__}")
        try:
            info = session(a).get("/api/v1/master")
            print(f"master: {info.get('version')} ({a.master}, cluster {info.get('cluster_id')})")
        except Exception as e:  # noqa: BLE001 -- the client version is still useful without a master
            print(f"master: unreachable at {a.master} ({e})")

    sub.add_parser("version").set_defaults(fn=version)

    def auth_token(a):
        tok = session(a).token
        if not tok:
            raise SystemExit("not logged in (det user login)")
        print(tok)

    def curl(a):
        s = session(a)
        body = json.loads(a.data) if a.data else None
        print(json.dumps(s.request(a.x.upper(), a.path, body=body), indent=2, default=str))

    def bindings_list(a):
        for r in session(a).get("/api/v1/_routes")["routes"]:
            print(f"{r['method']:6s} {r['path']}")

    def bindings_call(a):  # reference cli/dev.py `det dev bindings call`: one REST route by method + path
        s = session(a)
        body = json.loads(a.body) if a.body else None
        params = dict(kv.split("=", 1) for kv in a.param or [])
        print(json.dumps(s.request(a.method.upper(), a.path, body=body, params=params or None), indent=2, default=str))

    dv = sub.add_parser("dev").add_subparsers(dest="verb", required=True)
    _add(dv, "auth-token", auth_token)
    _add(dv, "curl", curl, "path", (("-X",), {"dest": "x", "default": "GET"}), (("-d", "--data"), {"default": None}))
    bd = dv.add_parser("bindings", aliases=["b"]).add_subparsers(dest="bverb", required=True)
    _add(bd, "list", bindings_list)
    _add(bd, "call", bindings_call, "method", "path", (("--body",), {"default": None}),
         (("-p", "--param"), {"action": "append", "default": None}))

    # ---------------------------------------------------------------- preview-search
    def preview(a):
        from determined_amd import config as expconf
        from determined_amd.searcher import simulate

        cfg = expconf.parse(_yaml_file(a.config_file))
        rng = random.Random(0)
        out = simulate(cfg["searcher"], cfg.get("hyperparameters", {}), lambda hp, length: rng.random(),
                       seed=int(cfg["reproducibility"]["experiment_seed"]))
        trials = out["trials"]
        unit = next(iter(cfg["searcher"].get("max_length") or {"batches": 0}))
        by_len: Dict[int, int] = {}
        for t in trials.values():
            by_len[t["trained"]] = by_len.get(t["trained"], 0) + 1
        print(f"Using search configuration: {cfg['searcher']['name']}")
        print(f"This search will create a total of {len(trials)} trial(s):")
        for length, n in sorted(by_len.items()):
            print(f"  {n} trial(s) trained for {length} {unit}")
        print(f"Total: {sum(t['trained'] for t in trials.values())} {unit}")

    _add(sub, "preview-search", preview, "config_file")


def _merge(dst: Dict[str, Any], src: Dict[str, Any]) -> None:
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = v
