"""``det`` command line interface (reference: ``harness/determined/cli`` + ``deploy/local``).

    python -m determined_amd.cli [-m MASTER] <noun> <verb> ...
"""

import argparse
import base64
import io
import json
import os
import pathlib
import signal
import subprocess
import sys
import tarfile
import time
from typing import Any, Dict, List, Optional

import yaml
from tabulate import tabulate

from determined_amd.common.api import APIException, Session

TERMINAL = {"COMPLETED", "CANCELED", "ERROR", "DELETED"}


def _session(a: argparse.Namespace) -> Session:
    from determined_amd.cli._iam import stored_token

    return Session(a.master, token=os.environ.get("DET_MASTER_TOKEN") or stored_token(a.master))


def _print(rows: List[Dict[str, Any]], cols: List[str], a: argparse.Namespace) -> None:
    if getattr(a, "json", False):
        print(json.dumps(rows, indent=2, default=str))
        return
    print(tabulate([[r.get(c) for c in cols] for r in rows], headers=cols))


def tar_model_dir(model_dir: str, includes: Optional[List[str]] = None) -> bytes:
    """gzip tar of the model definition (a directory or a single file) plus ``includes``
    (``det e create -i``: extra files / directories, added under their base names)."""
    root = pathlib.Path(model_dir)
    if root.is_file():
        buf = io.BytesIO()
        with tarfile.open(fileobj=buf, mode="w:gz") as tf:
            tf.add(root, arcname=root.name)
            for inc in includes or []:
                tf.add(inc, arcname=pathlib.Path(inc).name)
        return buf.getvalue()
    ignore = set()
    dignore = root / ".detignore"
    if dignore.exists():
        ignore = {ln.strip() for ln in dignore.read_text().splitlines() if ln.strip() and not ln.startswith("#")}
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w:gz") as tf:
        for p in sorted(root.rglob("*")):
            rel = p.relative_to(root)
            if any(part in ("__pycache__", ".git") for part in rel.parts) or any(rel.match(g) for g in ignore):
                continue
            tf.add(p, arcname=str(rel), recursive=False)
        for inc in includes or []:
            tf.add(inc, arcname=pathlib.Path(inc).name)
    data = buf.getvalue()
    if len(data) > 96 * 1024 * 1024:
        raise SystemExit("model definition directory is larger than 96 MiB; add a .detignore")
    return data


# ------------------------------------------------------------------------------------ experiments
def exp_create(a: argparse.Namespace) -> None:
    cfg = yaml.safe_load(open(a.config_file))
    if a.config:
        for kv in a.config:
            k, _, v = kv.partition("=")
            cur = cfg
            parts = k.split(".")
            for p in parts[:-1]:
                cur = cur.setdefault(p, {})
            cur[parts[-1]] = yaml.safe_load(v)
    if a.test:
        cfg["searcher"] = {"name": "single", "metric": cfg.get("searcher", {}).get("metric", "loss"),
                           "max_length": {"batches": 1}}
        cfg["max_restarts"] = 0
    if a.local:
        return _exp_local(cfg, a)
    s = _session(a)
    body: Dict[str, Any] = {"config": cfg, "activate": not a.paused}
    if a.model_def is not None:
        body["model_def"] = base64.b64encode(tar_model_dir(a.model_def, a.include)).decode()
    if a.template:
        body["template"] = a.template
    if a.project_id is not None:
        body["project_id"] = a.project_id
    r = s.post("/api/v1/experiments", body)
    eid = r["experiment"]["id"]
    print(f"Created experiment {eid}")
    if a.follow_first_trial or a.test:
        _follow_first_trial(s, eid)
        exp = s.get(f"/api/v1/experiments/{eid}")["experiment"]
        if a.test and exp["state"] != "COMPLETED":
            raise SystemExit(f"test experiment {eid} ended in state {exp['state']}")


def _exp_local(cfg: Dict[str, Any], a: argparse.Namespace) -> None:
    """Run the first trial of an experiment locally (no master) -- ``det e create --local``."""
    from determined_amd import config as expconf
    from determined_amd.searcher import decode_sample, flatten_hparams
    import random as _r

    cfg = expconf.parse(cfg)
    flat, tables = flatten_hparams(cfg["hyperparameters"])
    hp = decode_sample([(f["path"], 2, 0, 0.0) if f["type"] in (0, 4) else
                        (f["path"], 1, 0, (f["minval"] + f["maxval"]) / 2) for f in flat], tables)
    env = dict(os.environ)
    env.update(DET_LOCAL_HPARAMS=json.dumps(hp), DET_LOCAL_CONFIG=json.dumps(cfg))
    ep = cfg.get("entrypoint")
    code = subprocess.call([sys.executable, "-m", "determined_amd.exec.local", ep], cwd=a.model_def or ".", env=env)
    raise SystemExit(code)


def _follow_first_trial(s: Session, eid: int) -> None:
    tid = None
    while tid is None:
        trials = s.get(f"/api/v1/experiments/{eid}/trials")["trials"]
        if trials:
            tid = trials[0]["id"]
            break
        if s.get(f"/api/v1/experiments/{eid}")["experiment"]["state"] in TERMINAL:
            return
        time.sleep(0.5)
    _follow_logs(s, f"trial-{tid}", lambda: s.get(f"/api/v1/trials/{tid}")["trial"]["state"] in
                 ("COMPLETED", "CANCELED", "ERROR") or
                 s.get(f"/api/v1/experiments/{eid}")["experiment"]["state"] in TERMINAL)


def _follow_logs(s: Session, task_id: str, done) -> None:
    after = 0
    while True:
        logs = s.get(f"/api/v1/tasks/{task_id}/logs", params={"after": after})["logs"]
        for ln in logs:
            print(ln["log"])
            after = ln["id"]
        if not logs:
            if done():
                logs = s.get(f"/api/v1/tasks/{task_id}/logs", params={"after": after})["logs"]
                for ln in logs:
                    print(ln["log"])
                return
            time.sleep(0.5)


def exp_list(a):
    _print(_session(a).get("/api/v1/experiments")["experiments"],
           ["id", "name", "state", "progress", "num_trials", "searcher_type", "archived"], a)


def exp_describe(a):
    s = _session(a)
    r = s.get(f"/api/v1/experiments/{a.id}")
    if a.json:
        r["trials"] = s.get(f"/api/v1/experiments/{a.id}/trials")["trials"]
        print(json.dumps(r, indent=2, default=str))
        return
    e = r["experiment"]
    print(tabulate([[e["id"], e["name"], e["state"], f"{100 * (e['progress'] or 0):.1f}%", e["searcher_type"]]],
                   headers=["id", "name", "state", "progress", "searcher"]))
    trials = s.get(f"/api/v1/experiments/{a.id}/trials")["trials"]
    print()
    print(tabulate([[t["id"], t["state"], t["total_batches"], t["searcher_metric"], t["best_validation"],
                     t["restarts"], json.dumps(t["hparams"])[:80]] for t in trials],
                   headers=["trial", "state", "batches", "searcher metric", "best val", "restarts", "hparams"]))


def _simple(path: str, method: str = "post"):
    def fn(a):
        getattr(_session(a), method)(path.format(id=a.id))
        print("ok")

    return fn


def exp_wait(a):
    s = _session(a)
    while True:
        st = s.get(f"/api/v1/experiments/{a.id}")["experiment"]["state"]
        if st in TERMINAL:
            print(st)
            raise SystemExit(0 if st == "COMPLETED" else 1)
        time.sleep(a.polling_interval)


def exp_logs(a):
    s = _session(a)
    trials = s.get(f"/api/v1/experiments/{a.id}/trials")["trials"]
    if not trials:
        raise SystemExit("experiment has no trials yet")
    a.trial_id = trials[0]["id"]
    trial_logs(a)


def exp_checkpoints(a):
    rows = _session(a).get(f"/api/v1/experiments/{a.id}/checkpoints")["checkpoints"]
    if a.best is not None:
        rows = sorted([r for r in rows if r.get("searcher_metric") is not None and r["state"] == "COMPLETED"],
                      key=lambda r: r["searcher_metric"])[: a.best]
    _print(rows, ["uuid", "trial_id", "steps_completed", "state", "searcher_metric"], a)


def exp_trials(a):
    _print(_session(a).get(f"/api/v1/experiments/{a.id}/trials")["trials"],
           ["id", "state", "total_batches", "searcher_metric", "best_validation", "restarts"], a)


# ------------------------------------------------------------------------------------ trials
def trial_describe(a):
    s = _session(a)
    t = s.get(f"/api/v1/trials/{a.id}")["trial"]
    if a.json:
        t["metrics"] = s.get(f"/api/v1/trials/{a.id}/metrics")["metrics"]
        print(json.dumps(t, indent=2, default=str))
        return
    print(tabulate([[t["id"], t["experiment_id"], t["state"], t["total_batches"], t["latest_checkpoint"],
                     json.dumps(t["hparams"])]], headers=["trial", "experiment", "state", "batches", "checkpoint",
                                                          "hparams"]))
    if a.metrics:
        ms = s.get(f"/api/v1/trials/{a.id}/metrics")["metrics"]
        print(tabulate([[m["group_name"], m["steps_completed"], json.dumps(m["metrics"])] for m in ms],
                       headers=["group", "steps", "metrics"]))


def trial_logs(a):
    s = _session(a)
    tid = getattr(a, "trial_id", None) or a.id
    if a.follow:
        _follow_logs(s, f"trial-{tid}", lambda: s.get(f"/api/v1/trials/{tid}")["trial"]["state"] in
                     ("COMPLETED", "CANCELED", "ERROR"))
        return
    for ln in s.get(f"/api/v1/tasks/trial-{tid}/logs")["logs"]:
        print(ln["log"])


def trial_checkpoints(a):
    _print(_session(a).get(f"/api/v1/trials/{a.id}/checkpoints")["checkpoints"],
           ["uuid", "steps_completed", "state", "searcher_metric"], a)


# ------------------------------------------------------------------------------------ checkpoints
def ckpt_describe(a):
    c = _session(a).get(f"/api/v1/checkpoints/{a.uuid}")["checkpoint"]
    print(json.dumps(c, indent=2, default=str))


def ckpt_download(a):
    from determined_amd import storage

    c = _session(a).get(f"/api/v1/checkpoints/{a.uuid}")["checkpoint"]
    if not c.get("checkpoint_storage"):
        raise SystemExit("checkpoint storage unknown for this checkpoint")
    out = a.output_dir or os.path.join("checkpoints", a.uuid)
    storage.build(c["checkpoint_storage"]).download(a.uuid, out)
    print(out)


def ckpt_delete(a):
    s = _session(a)
    for u in a.uuids:
        s.delete(f"/api/v1/checkpoints/{u}")
    print("ok")


# ------------------------------------------------------------------------------------ models
def model_create(a):
    m = _session(a).post("/api/v1/models", {"name": a.name, "description": a.description or ""})["model"]
    print(f"Created model {m['name']} (id {m['id']})")


def model_list(a):
    _print(_session(a).get("/api/v1/models")["models"], ["id", "name", "description", "creation_time"], a)


def model_describe(a):
    s = _session(a)
    m = s.get(f"/api/v1/models/{a.name}")["model"]
    v = s.get(f"/api/v1/models/{a.name}/versions")["model_versions"]
    if a.json:
        print(json.dumps({"model": m, "versions": v}, indent=2, default=str))
        return
    print(tabulate([[m["id"], m["name"], m["description"]]], headers=["id", "name", "description"]))
    print(tabulate([[x["version"], x["checkpoint_uuid"], x["name"]] for x in v], headers=["version", "checkpoint",
                                                                                            "name"]))


def model_register(a):
    v = _session(a).post(f"/api/v1/models/{a.name}/versions", {"checkpoint_uuid": a.uuid})["model_version"]
    print(f"Registered checkpoint {a.uuid} as version {v['version']} of {a.name}")


# ------------------------------------------------------------------------------------ cluster
def master_info(a):
    print(json.dumps(_session(a).get("/api/v1/master"), indent=2))


def agent_list(a):
    _print(_session(a).get("/api/v1/agents")["agents"], ["id", "host", "slots", "used_slots", "gpu", "enabled"], a)


def slot_list(a):
    rows = []
    for ag in _session(a).get("/api/v1/agents")["agents"]:
        disabled = set(ag.get("disabled_slots") or [])
        for i, owner in enumerate(ag["slot_owner"]):
            rows.append({"agent": ag["id"], "slot": i, "device": ag["devices"][i] if i < len(ag["devices"]) else i,
                         "type": "rocm" if ag["gpu"] else "cpu", "enabled": i not in disabled and ag["enabled"],
                         "allocation": owner or ""})
    _print(rows, ["agent", "slot", "device", "type", "enabled", "allocation"], a)


def pool_list(a):
    _print(_session(a).get("/api/v1/resource-pools")["resource_pools"],
           ["name", "scheduler_type", "slots_available", "slots_used", "num_agents"], a)


def job_list(a):
    _print(_session(a).get("/api/v1/job-queues")["jobs"],
           ["alloc_id", "job_id", "slots", "priority", "allocated", "preempting"], a)


def cmd_run(a):
    s = _session(a)
    r = s.post("/api/v1/commands", {"command": " ".join(a.cmd), "slots": a.slots,
                                    "resource_pool": getattr(a, "resource_pool", None),
                                    "priority": getattr(a, "priority", None),
                                    "template": getattr(a, "template", None)})
    print(f"Launched command {r['task_id']}")
    if not a.detach:
        _follow_logs(s, r["task_id"], lambda: s.get(f"/api/v1/tasks/{r['task_id']}")["task"]["state"] in
                     ("TERMINATED", "CANCELED"))


def task_list(a):
    _print(_session(a).get("/api/v1/tasks")["tasks"], ["id", "type", "state", "exit_code"], a)


def task_logs(a):
    for ln in _session(a).get(f"/api/v1/tasks/{a.task_id}/logs")["logs"]:
        print(ln["log"])


def template_set(a):
    _session(a).request("PUT", f"/api/v1/templates/{a.name}", body={"config": yaml.safe_load(open(a.file))})
    print("ok")


def template_list(a):
    _print(_session(a).get("/api/v1/templates")["templates"], ["name"], a)


def webhook_create(a):
    w = _session(a).post("/api/v1/webhooks", {"url": a.url, "triggers": a.trigger or []})["webhook"]
    print(f"Created webhook {w['id']}")


def webhook_list(a):
    _print(_session(a).get("/api/v1/webhooks")["webhooks"], ["id", "url", "triggers"], a)


# ------------------------------------------------------------------------------------ deploy local
def _local_dir() -> pathlib.Path:
    d = pathlib.Path(os.environ.get("DET_LOCAL_CLUSTER_DIR", os.path.expanduser("~/.local/share/determined_amd/local")))
    d.mkdir(parents=True, exist_ok=True)
    return d


def _pids() -> Dict[str, int]:
    f = _local_dir() / "pids.json"
    return json.loads(f.read_text()) if f.exists() else {}


def _save_pids(pids: Dict[str, int]) -> None:
    f = _local_dir() / "pids.json"
    if pids:
        f.write_text(json.dumps(pids))
    elif f.exists():
        f.unlink()


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except (ProcessLookupError, PermissionError):
        return False


def _stop(pids: Dict[str, int], name: str) -> None:
    pid = pids.pop(name, None)
    if pid is None:
        return
    try:
        os.killpg(pid, signal.SIGTERM)
    except ProcessLookupError:
        pass


def _start_master(a, pids: Dict[str, int]) -> str:
    """``det deploy local master-up`` (reference deploy/local/cli.py): the master as a local process
    (sqlite db + logs under the local cluster directory)."""
    d = _local_dir()
    if "master" in pids and _alive(pids["master"]):
        raise SystemExit(f"a local master is already running (pid {pids['master']}); run `det deploy local master-down`")
    port = a.master_port
    cmd = [sys.executable, "-m", "determined_amd.master", "--port", str(port), "--db", str(d / "master.db"),
           "--scheduler", a.scheduler]
    if getattr(a, "master_config_path", None):
        cmd += ["--config-file", str(a.master_config_path)]
    mlog = open(d / "master.log", "a")
    mp = subprocess.Popen(cmd, stdout=mlog, stderr=subprocess.STDOUT, env=dict(os.environ), start_new_session=True)
    pids["master"] = mp.pid
    url = f"http://127.0.0.1:{port}"
    s = Session(url, max_retries=0)
    for _ in range(100):
        try:
            s.get("/api/v1/master")
            break
        except Exception:
            if mp.poll() is not None:
                raise SystemExit(f"the master exited (code {mp.returncode}); see {d / 'master.log'}")
            time.sleep(0.2)
    return url


def _start_agent(name: str, url: str, a, pids: Dict[str, int]) -> None:
    d = _local_dir()
    key = f"agent-{name}" if not name.startswith("agent-") else name
    if key in pids and _alive(pids[key]):
        raise SystemExit(f"agent {key} is already running (pid {pids[key]})")
    alog = open(d / f"{key}.log", "a")
    cmd = [sys.executable, "-m", "determined_amd.agent", "--master-url", url, "--agent-id", key]
    if a.no_gpu:
        cmd += ["--slots", str(a.cpu_slots)]
    if getattr(a, "resource_pool", None):
        cmd += ["--resource-pool", a.resource_pool]
    ap = subprocess.Popen(cmd, stdout=alog, stderr=subprocess.STDOUT, env=dict(os.environ), start_new_session=True)
    pids[key] = ap.pid


def cluster_up(a):
    pids = _pids()
    if any(_alive(p) for p in pids.values()):
        raise SystemExit(f"a local cluster seems to be running ({_local_dir() / 'pids.json'}); "
                         "run `det deploy local cluster-down`")
    pids = {}
    url = _start_master(a, pids)
    for i in range(a.agents):
        _start_agent(str(i), url, a, pids)
    _save_pids(pids)
    print(f"local cluster up: master {url}, {a.agents} agent(s); logs in {_local_dir()}")


def cluster_down(a):
    pids = _pids()
    if not pids:
        print("no local cluster running")
        return
    for name in list(pids):
        _stop(pids, name)
    _save_pids(pids)
    print("local cluster down")


def master_up(a):
    pids = _pids()
    url = _start_master(a, pids)
    _save_pids(pids)
    print(f"local master up: {url}; logs in {_local_dir() / 'master.log'}")


def master_down(a):
    pids = _pids()
    if "master" not in pids:
        print("no local master running")
        return
    _stop(pids, "master")
    _save_pids(pids)
    print("local master down")


def agent_up(a):
    pids = _pids()
    name = a.agent_name or f"{len([k for k in pids if k.startswith('agent-')])}"
    _start_agent(name, a.master_url or a.master, a, pids)
    _save_pids(pids)
    print(f"local agent {name} up (master {a.master_url or a.master})")


def agent_down(a):
    pids = _pids()
    names = [k for k in pids if k.startswith("agent-")] if a.all else \
        [a.agent_name if a.agent_name.startswith("agent-") else f"agent-{a.agent_name}"]
    for n in names:
        _stop(pids, n)
    _save_pids(pids)
    print(f"stopped {', '.join(names) or 'no agents'}")


def local_logs(a):
    """``det deploy local logs``: the local master's log (follows unless --no-follow)."""
    f = _local_dir() / (f"agent-{a.agent_name}.log" if a.agent_name else "master.log")
    if not f.exists():
        raise SystemExit(f"no log at {f}")
    with open(f) as fh:
        sys.stdout.write(fh.read())
        sys.stdout.flush()
        while not a.no_follow:
            line = fh.readline()
            if line:
                sys.stdout.write(line)
                sys.stdout.flush()
            else:
                time.sleep(0.5)


# ------------------------------------------------------------------------------------ parser
def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="det", description="determined_amd CLI")
    p.add_argument("-m", "--master", default=os.environ.get("DET_MASTER", "http://127.0.0.1:8080"))
    p.add_argument("--json", action="store_true")
    sub = p.add_subparsers(dest="noun", required=True)

    e = sub.add_parser("experiment", aliases=["e"]).add_subparsers(dest="verb", required=True)
    c = e.add_parser("create")
    c.add_argument("config_file")
    c.add_argument("model_def", nargs="?", default=None)
    c.add_argument("-i", "--include", action="append", default=[], help="extra files to ship with the model")
    c.add_argument("--template", default=None, help="template to apply to the experiment config")
    c.add_argument("--project_id", "--project-id", type=int, default=None, dest="project_id")
    c.add_argument("--paused", action="store_true")
    c.add_argument("-f", "--follow-first-trial", action="store_true")
    c.add_argument("-t", "--test", "--test-mode", action="store_true", dest="test")
    c.add_argument("--local", action="store_true")
    c.add_argument("--config", action="append", help="override: key.sub=value")
    c.set_defaults(fn=exp_create)
    e.add_parser("list").set_defaults(fn=exp_list)
    for verb, fn in (("describe", exp_describe), ("wait", exp_wait), ("logs", exp_logs),
                     ("list-trials", exp_trials),
                     ("pause", _simple("/api/v1/experiments/{id}/pause")),
                     ("activate", _simple("/api/v1/experiments/{id}/activate")),
                     ("kill", _simple("/api/v1/experiments/{id}/kill")),
                     ("cancel", _simple("/api/v1/experiments/{id}/cancel")),
                     ("archive", _simple("/api/v1/experiments/{id}/archive")),
                     ("unarchive", _simple("/api/v1/experiments/{id}/unarchive")),
                     ("delete", _simple("/api/v1/experiments/{id}", "delete"))):
        sp = e.add_parser(verb)
        sp.add_argument("id", type=int)
        if verb == "wait":
            sp.add_argument("--polling-interval", type=float, default=2.0)
        if verb == "logs":
            sp.add_argument("-f", "--follow", action="store_true")
        sp.set_defaults(fn=fn)
    lc = e.add_parser("list-checkpoints")
    lc.add_argument("id", type=int)
    lc.add_argument("--best", type=int, default=None)
    lc.set_defaults(fn=exp_checkpoints)

    t = sub.add_parser("trial", aliases=["t"]).add_subparsers(dest="verb", required=True)
    td = t.add_parser("describe")
    td.add_argument("id", type=int)
    td.add_argument("--metrics", action="store_true")
    td.set_defaults(fn=trial_describe)
    tl = t.add_parser("logs")
    tl.add_argument("id", type=int)
    tl.add_argument("-f", "--follow", action="store_true")
    tl.set_defaults(fn=trial_logs)
    tk = t.add_parser("kill")
    tk.add_argument("id", type=int)
    tk.set_defaults(fn=_simple("/api/v1/trials/{id}/kill"))
    tc = t.add_parser("list-checkpoints")
    tc.add_argument("id", type=int)
    tc.set_defaults(fn=trial_checkpoints)

    ck = sub.add_parser("checkpoint", aliases=["c"]).add_subparsers(dest="verb", required=True)
    cd = ck.add_parser("describe")
    cd.add_argument("uuid")
    cd.set_defaults(fn=ckpt_describe)
    cdl = ck.add_parser("download")
    cdl.add_argument("uuid")
    cdl.add_argument("-o", "--output-dir", default=None)
    cdl.set_defaults(fn=ckpt_download)
    cdel = ck.add_parser("delete")
    cdel.add_argument("uuids", nargs="+")
    cdel.set_defaults(fn=ckpt_delete)

    mo = sub.add_parser("model", aliases=["m"]).add_subparsers(dest="verb", required=True)
    mc = mo.add_parser("create")
    mc.add_argument("name")
    mc.add_argument("--description", default="")
    mc.set_defaults(fn=model_create)
    mo.add_parser("list").set_defaults(fn=model_list)
    md = mo.add_parser("describe")
    md.add_argument("name")
    md.set_defaults(fn=model_describe)
    mr = mo.add_parser("register-version")
    mr.add_argument("name")
    mr.add_argument("uuid")
    mr.set_defaults(fn=model_register)

    from determined_amd.cli import _ntsc

    master_fns = _ntsc.register(sub, _session, _print, _follow_logs)
    ms = sub.add_parser("master").add_subparsers(dest="verb", required=True)
    ms.add_parser("info").set_defaults(fn=master_info)
    ms.add_parser("config").set_defaults(fn=master_fns["config"])
    ml = ms.add_parser("logs")
    ml.add_argument("--tail", type=int, default=200)
    ml.set_defaults(fn=master_fns["logs"])
    sub.add_parser("agent", aliases=["a"]).add_subparsers(dest="verb", required=True).add_parser(
        "list").set_defaults(fn=agent_list)
    sub.add_parser("slot", aliases=["s"]).add_subparsers(dest="verb", required=True).add_parser(
        "list").set_defaults(fn=slot_list)
    sub.add_parser("resource-pool", aliases=["rp"]).add_subparsers(dest="verb", required=True).add_parser(
        "list").set_defaults(fn=pool_list)
    jb = sub.add_parser("job", aliases=["j"]).add_subparsers(dest="verb", required=True)
    jb.add_parser("list").set_defaults(fn=job_list)

    cm = sub.add_parser("command", aliases=["cmd"]).add_subparsers(dest="verb", required=True)
    cm.add_parser("list").set_defaults(fn=lambda a: _print(_session(a).get("/api/v1/commands")["tasks"],
                                                           ["id", "type", "state", "exit_code"], a))
    ck_ = cm.add_parser("kill")
    ck_.add_argument("task_id")
    ck_.set_defaults(fn=lambda a: _session(a).post(f"/api/v1/tasks/{a.task_id}/kill", {}))
    cr = cm.add_parser("run")
    cr.add_argument("cmd", nargs=argparse.REMAINDER)
    cr.add_argument("--slots", type=int, default=None)
    cr.add_argument("--template", default=None, help="template to apply to the command config")
    cr.add_argument("-d", "--detach", action="store_true")
    cr.set_defaults(fn=cmd_run)

    tk2 = sub.add_parser("task").add_subparsers(dest="verb", required=True)
    tk2.add_parser("list").set_defaults(fn=task_list)
    tlg = tk2.add_parser("logs")
    tlg.add_argument("task_id")
    tlg.set_defaults(fn=task_logs)

    from determined_amd.cli import _extra

    _extra.register({"experiment": e, "trial": t, "model": mo, "job": jb, "task": tk2}, _session, _print)

    tp = sub.add_parser("template", aliases=["tpl"]).add_subparsers(dest="verb", required=True)
    _extra.register_template(tp, _session)
    ts = tp.add_parser("set")
    ts.add_argument("name")
    ts.add_argument("file")
    ts.set_defaults(fn=template_set)
    tp.add_parser("list").set_defaults(fn=template_list)

    wh = sub.add_parser("webhook").add_subparsers(dest="verb", required=True)
    wc = wh.add_parser("create")
    wc.add_argument("url")
    wc.add_argument("--trigger", action="append")
    wc.set_defaults(fn=webhook_create)
    wh.add_parser("list").set_defaults(fn=webhook_list)

    from determined_amd.cli import _iam

    _iam.register(sub, _session, _print)
    _iam.register_experiment_move(e, _session)

    from determined_amd.cli import _more

    _more.register(sub, _session, _print, _follow_logs)

    dp = sub.add_parser("deploy").add_subparsers(dest="where", required=True)
    loc = dp.add_parser("local").add_subparsers(dest="verb", required=True)
    up = loc.add_parser("cluster-up")
    up.add_argument("--master-port", type=int, default=8080)
    up.add_argument("--master-config-path", default=None, help="master configuration (YAML)")
    up.add_argument("--agents", type=int, default=1)
    up.add_argument("--no-gpu", action="store_true")
    up.add_argument("--cpu-slots", type=int, default=8)
    up.add_argument("--scheduler", default="priority", choices=["priority", "fair_share", "round_robin"])
    up.set_defaults(fn=cluster_up)
    loc.add_parser("cluster-down").set_defaults(fn=cluster_down)
    mu = loc.add_parser("master-up")
    mu.add_argument("--master-port", type=int, default=8080)
    mu.add_argument("--master-config-path", default=None)
    mu.add_argument("--scheduler", default="priority", choices=["priority", "fair_share", "round_robin"])
    mu.set_defaults(fn=master_up)
    loc.add_parser("master-down").set_defaults(fn=master_down)
    au = loc.add_parser("agent-up")
    au.add_argument("master_url", nargs="?", default=None)
    au.add_argument("--agent-name", default=None)
    au.add_argument("--no-gpu", action="store_true")
    au.add_argument("--cpu-slots", type=int, default=8)
    au.add_argument("--resource-pool", default=None)
    au.set_defaults(fn=agent_up)
    ad = loc.add_parser("agent-down")
    ad.add_argument("--agent-name", default="0")
    ad.add_argument("--all", action="store_true")
    ad.set_defaults(fn=agent_down)
    lg = loc.add_parser("logs")
    lg.add_argument("--no-follow", action="store_true")
    lg.add_argument("--agent-name", default=None)
    lg.set_defaults(fn=local_logs)
    return p


def main(argv: Optional[List[str]] = None) -> int:
    a = build_parser().parse_args(argv)
    try:
        a.fn(a)
    except APIException as e:
        print(f"Error: {e}", file=sys.stderr)
        return 1
    return 0
