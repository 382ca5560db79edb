"""``det notebook|shell|tensorboard|command`` and ``det master config|logs`` (reference:
``harness/determined/cli/{notebook,shell,tensorboard,command,master}.py``)."""

import argparse
import json
import os
import shlex
import socket
import subprocess
import sys
import time
from typing import Any, Dict

LOCAL_HOSTS = {"127.0.0.1", "localhost", "::1"}


def _wait_proxy(s: Any, task_id: str, timeout: float = 120.0) -> Dict[str, Any]:
    t0 = time.time()
    while time.time() - t0 < timeout:
        t = s.get(f"/api/v1/tasks/{task_id}")["task"]
        if t.get("proxy"):
            return t
        if t["state"] in ("TERMINATED", "CANCELED"):
            logs = "\n".join(ln["log"] for ln in s.get(f"/api/v1/tasks/{task_id}/logs")["logs"][-20:])
            raise SystemExit(f"task {task_id} ended before it was ready (exit {t.get('exit_code')}):\n{logs}")
        time.sleep(0.3)
    raise SystemExit(f"task {task_id} not ready after {timeout:.0f}s")


def _is_local(host: str) -> bool:
    if host in LOCAL_HOSTS:
        return True
    try:
        return host in {socket.gethostbyname(socket.gethostname()), socket.gethostname()}
    except OSError:
        return False


def shell_command(task: Dict[str, Any]) -> Dict[str, Any]:
    """argv + env for an interactive shell inside the task's allocation."""
    px = task["proxy"]
    env = dict(px.get("env") or {})
    if _is_local(px["host"]):
        return {"argv": ["bash", "-i"], "env": env, "cwd": px.get("cwd")}
    exports = " ".join(f"{k}={shlex.quote(v)}" for k, v in env.items())
    remote = f"cd {shlex.quote(px.get('cwd') or '~')} && env {exports} bash -i"
    return {"argv": ["ssh", "-t", px["host"], remote], "env": {}, "cwd": None}


def _pool_args(a: Any) -> Dict[str, Any]:
    """--resource-pool / --priority (added by cli/_more.py to every task-creating verb)."""
    return {k: getattr(a, k, None) for k in ("resource_pool", "priority")}


def register(sub: Any, session: Any, show: Any, follow_logs: Any) -> None:
    cols = ["id", "type", "state", "exit_code"]

    def lister(plural):
        def fn(a):
            show(session(a).get(f"/api/v1/{plural}")["tasks"], cols, a)
        return fn

    def killer(a):
        session(a).post(f"/api/v1/tasks/{a.task_id}/kill", {})
        print(f"killed {a.task_id}")

    def logs(a):
        for ln in session(a).get(f"/api/v1/tasks/{a.task_id}/logs")["logs"]:
            print(ln["log"])

    def common(p, plural, start_fn, extra=()):
        g = p.add_subparsers(dest="verb", required=True)
        st = g.add_parser("start")
        for args, kw in extra:
            st.add_argument(*args, **kw)
        st.set_defaults(fn=start_fn)
        g.add_parser("list").set_defaults(fn=lister(plural))
        for verb, fn in (("kill", killer), ("logs", logs)):
            k = g.add_parser(verb)
            k.add_argument("task_id")
            k.set_defaults(fn=fn)
        return g

    # ---------------------------------------------------------------- tensorboard
    def tb_start(a):
        s = session(a)
        r = s.post("/api/v1/tensorboards", {"experiment_ids": a.experiment_ids, "trial_ids": a.trial_id or [],
                                            **_pool_args(a)})
        t = _wait_proxy(s, r["task_id"])
        print(f"Launched tensorboard {r['task_id']}: http://{t['proxy']['host']}:{t['proxy']['port']}/")

    def tb_open(a):  # through the master's task proxy, as the reference (master/internal/proxy)
        t = session(a).get(f"/api/v1/tasks/{a.task_id}")["task"]
        print(f"{a.master.rstrip('/')}/proxy/{a.task_id}/" if t.get("proxy") else "not ready")

    g = common(sub.add_parser("tensorboard"), "tensorboards", tb_start,
               [(("experiment_ids",), {"type": int, "nargs": "*"}),
                (("-t", "--trial-id"), {"type": int, "action": "append"})])
    o = g.add_parser("open")
    o.add_argument("task_id")
    o.set_defaults(fn=tb_open)

    # ---------------------------------------------------------------- notebook
    def nb_start(a):
        s = session(a)
        r = s.post("/api/v1/notebooks", {"slots": a.slots, **_pool_args(a)})
        t = _wait_proxy(s, r["task_id"])
        print(f"Launched notebook {r['task_id']}: http://{t['proxy']['host']}:{t['proxy']['port']}/lab")

    def nb_open(a):
        t = session(a).get(f"/api/v1/tasks/{a.task_id}")["task"]
        print(f"{a.master.rstrip('/')}/proxy/{a.task_id}/lab" if t.get("proxy") else "not ready")

    nb = common(sub.add_parser("notebook"), "notebooks", nb_start, [(("--slots",), {"type": int, "default": 1})])
    o = nb.add_parser("open")
    o.add_argument("task_id")
    o.set_defaults(fn=nb_open)

    # ---------------------------------------------------------------- shell
    def sh_start(a):
        s = session(a)
        r = s.post("/api/v1/shells", {"slots": a.slots, "idle_timeout": a.idle_timeout, **_pool_args(a)})
        _wait_proxy(s, r["task_id"])
        print(f"Launched shell {r['task_id']}")
        if not a.detach:
            a.task_id = r["task_id"]
            sh_open(a)

    def sh_open(a):
        s = session(a)
        t = _wait_proxy(s, a.task_id)
        if (t.get("proxy") or {}).get("tunnel"):  # the task's PTY server, through the master
            from determined_amd.cli import _tunnel

            cmd = [c for c in (getattr(a, "command", None) or []) if c != "--"]
            sys.exit(_tunnel.run(s.master_url, a.task_id, cmd or None, token=s.token))
        sc = shell_command(t)
        env = dict(os.environ)
        env.update(sc["env"])
        rc = subprocess.call(sc["argv"], env=env, cwd=sc["cwd"] if sc["cwd"] and os.path.isdir(sc["cwd"]) else None)
        sys.exit(rc)

    def sh_ssh(a):
        t = _wait_proxy(session(a), a.task_id)
        if (t.get("proxy") or {}).get("tunnel"):
            print(f"det -m {a.master} shell open {a.task_id}   # tunnelled through the master, no ssh needed")
            return
        sc = shell_command(t)
        print(shlex.join(sc["argv"]) if sc["argv"][0] == "ssh" else
              " ".join(f"{k}={shlex.quote(v)}" for k, v in sc["env"].items()) + " bash -i")

    g = common(sub.add_parser("shell"), "shells", sh_start,
               [(("--slots",), {"type": int, "default": 1}), (("--idle-timeout",), {"type": float, "default": 0.0}),
                (("-d", "--detach"), {"action": "store_true"})])
    for verb, fn in (("open", sh_open), ("show-ssh-command", sh_ssh)):
        o = g.add_parser(verb)
        o.add_argument("task_id")
        if verb == "open":
            o.add_argument("command", nargs=argparse.REMAINDER, help="run this instead of a login shell")
        o.set_defaults(fn=fn)

    # ---------------------------------------------------------------- master config / logs
    def master_config(a):
        print(json.dumps(session(a).get("/api/v1/master/config")["config"], indent=2))

    def master_logs(a):
        for r in session(a).get("/api/v1/master/logs", params={"limit": a.tail})["logs"]:
            print(f"{time.strftime('%Y-%m-%d %H:%M:%S', time.localtime(r['ts']))} {r['level']} {r['logger']}: "
                  f"{r['message']}")

    return {"config": master_config, "logs": master_logs}
