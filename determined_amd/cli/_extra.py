"""Remaining ``det`` verbs of the reference CLI (``harness/determined/cli/{experiment,trial,
model,job,task,template}.py``): experiment config / download-model-def / continue / download /
label / set ... / delete-tb-files, trial download / support-bundle / set log-retention, model
list-versions / delete / move, job update-batch, task config / kill, template describe / remove."""

import base64
import json
import os
from typing import Any, Dict

import yaml


def _kv(pairs) -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    for p in pairs or []:
        k, _, v = p.partition("=")
        out[k] = yaml.safe_load(v)
    return out


def register(groups: Dict[str, Any], session: Any, show: Any) -> None:
    e, t, mo, jb, tk = groups["experiment"], groups["trial"], groups["model"], groups["job"], groups["task"]

    def add(group, name, fn, *args, **kw):
        p = group.add_parser(name, **kw)
        for a_ in args:
            if isinstance(a_, tuple):
                p.add_argument(*a_[0], **a_[1])
            else:
                p.add_argument(a_)
        p.set_defaults(fn=fn)
        return p

    # ---------------------------------------------------------------- experiment
    def exp_config(a):
        print(yaml.safe_dump(session(a).get(f"/api/v1/experiments/{a.id}")["config"], sort_keys=False), end="")

    def exp_model_def(a):
        b64 = session(a).get(f"/api/v1/experiments/{a.id}/model_def")["b64_tgz"]
        if not b64:
            raise SystemExit(f"experiment {a.id} has no model definition")
        out = a.output_dir and os.path.join(a.output_dir, f"experiment_{a.id}_model_def.tgz") or \
            f"experiment_{a.id}_model_def.tgz"
        with open(out, "wb") as f:
            f.write(base64.b64decode(b64))
        print(out)

    def exp_continue(a):
        r = session(a).post(f"/api/v1/experiments/{a.id}/continue", {"overrides": _kv(a.config)})
        print(f"Continued experiment {a.id} as experiment {r['experiment_id']}")

    def exp_download(a):
        from determined_amd import storage

        s = session(a)
        cfg = s.get(f"/api/v1/experiments/{a.id}")["config"]
        sib = cfg["searcher"].get("smaller_is_better", True)
        ck = [c for c in s.get(f"/api/v1/experiments/{a.id}/checkpoints")["checkpoints"] if c["state"] == "COMPLETED"]
        ck = [c for c in ck if c.get("searcher_metric") is not None] or ck
        ck.sort(key=lambda c: (c.get("searcher_metric") or 0.0) * (1 if sib else -1))
        sm = storage.build(cfg["checkpoint_storage"])
        for c in ck[: a.top_n]:
            out = os.path.join(a.output_dir or "checkpoints", c["uuid"])
            sm.download(c["uuid"], out)
            print(out)

    def exp_label(verb):
        def fn(a):
            r = session(a).post(f"/api/v1/experiments/{a.id}/labels", {verb: [a.label]})
            print(", ".join(r["labels"]))
        return fn

    def exp_set(field):
        def fn(a):
            s = session(a)
            v = getattr(a, "value", None)
            if field in ("description", "name"):
                s.patch(f"/api/v1/experiments/{a.id}", {field: v})
            elif field in ("max-slots", "weight", "priority"):
                key = field.replace("-", "_")
                val = None if (key == "max_slots" and str(v).lower() == "none") else (
                    float(v) if key == "weight" else int(v))
                s.post(f"/api/v1/experiments/{a.id}/resources", {key: val})
            elif field == "gc-policy":
                body = {k: int(getattr(a, k)) for k in ("save_experiment_best", "save_trial_best",
                                                          "save_trial_latest") if getattr(a, k) is not None}
                s.patch(f"/api/v1/experiments/{a.id}/config/checkpoint_storage", body)
            elif field == "log-retention":
                days = -1 if a.forever else int(a.days)
                s.patch(f"/api/v1/experiments/{a.id}/config/retention_policy", {"log_retention_days": days})
            print(f"experiment {a.id}: {field} updated")
        return fn

    def exp_delete_tb(a):
        r = session(a).delete(f"/api/v1/experiments/{a.id}/tensorboard-files")
        print("deleted" if r and r.get("deleted") else "no tensorboard files")

    ID = (("id",), {"type": int})
    add(e, "config", exp_config, ID)
    add(e, "download-model-def", exp_model_def, ID, (("--output-dir",), {"default": None}))
    add(e, "continue", exp_continue, ID, (("--config",), {"action": "append", "help": "dotted.key=value override"}))
    add(e, "download", exp_download, ID, (("--top-n",), {"type": int, "default": 1}),
        (("-o", "--output-dir"), {"default": None}))
    lab = e.add_parser("label").add_subparsers(dest="labverb", required=True)
    for verb in ("add", "remove"):
        add(lab, verb, exp_label(verb), ID, "label")
    st = e.add_parser("set").add_subparsers(dest="field", required=True)
    for field in ("description", "name", "max-slots", "weight", "priority"):
        add(st, field, exp_set(field), ID, "value")
    add(st, "gc-policy", exp_set("gc-policy"), ID, (("--save-experiment-best",), {"type": int, "default": None}),
        (("--save-trial-best",), {"type": int, "default": None}),
        (("--save-trial-latest",), {"type": int, "default": None}))
    add(st, "log-retention", exp_set("log-retention"), ID, (("--days",), {"type": int, "default": 30}),
        (("--forever",), {"action": "store_true"}))
    add(e, "delete-tb-files", exp_delete_tb, ID)

    # ---------------------------------------------------------------- trial
    def trial_download(a):
        from determined_amd import storage

        s = session(a)
        tr = s.get(f"/api/v1/trials/{a.id}")["trial"]
        cfg = s.get(f"/api/v1/experiments/{tr['experiment_id']}")["config"]
        ck = [c for c in s.get(f"/api/v1/trials/{a.id}/checkpoints")["checkpoints"] if c["state"] == "COMPLETED"]
        if not ck:
            raise SystemExit(f"trial {a.id} has no completed checkpoint")
        if a.latest:
            c = max(ck, key=lambda c: c.get("steps_completed") or 0)
        else:
            sib = cfg["searcher"].get("smaller_is_better", True)
            scored = [c for c in ck if c.get("searcher_metric") is not None] or ck
            c = sorted(scored, key=lambda c: (c.get("searcher_metric") or 0.0) * (1 if sib else -1))[0]
        out = os.path.join(a.output_dir or "checkpoints", c["uuid"])
        storage.build(cfg["checkpoint_storage"]).download(c["uuid"], out)
        print(out)

    def trial_bundle(a):
        r = session(a).get(f"/api/v1/trials/{a.id}/support-bundle")
        out = os.path.join(a.output_dir or ".", f"bundle-trial-{a.id}.tar.gz")
        with open(out, "wb") as f:
            f.write(base64.b64decode(r["b64_tgz"]))
        print(out)

    def trial_retention(a):
        session(a).patch(f"/api/v1/trials/{a.id}", {"log_retention_days": -1 if a.forever else a.days})

    add(t, "download", trial_download, ID, (("--latest",), {"action": "store_true"}),
        (("-o", "--output-dir"), {"default": None}))
    add(t, "support-bundle", trial_bundle, ID, (("-o", "--output-dir"), {"default": None}))
    tset = t.add_parser("set").add_subparsers(dest="field", required=True)
    add(tset, "log-retention", trial_retention, ID, (("--days",), {"type": int, "default": 30}),
        (("--forever",), {"action": "store_true"}))

    # ---------------------------------------------------------------- model
    def model_versions(a):
        show(session(a).get(f"/api/v1/models/{a.name}/versions")["model_versions"],
             ["version", "checkpoint_uuid", "name", "comment"], a)

    def model_delete(a):
        session(a).delete(f"/api/v1/models/{a.name}")

    def model_move(a):
        session(a).patch(f"/api/v1/models/{a.name}", {"workspace": a.workspace})

    add(mo, "list-versions", model_versions, "name")
    add(mo, "delete", model_delete, "name")
    add(mo, "move", model_move, "name", "workspace")

    # ---------------------------------------------------------------- job / task
    def job_update(a):
        ups = []
        for spec in a.updates:  # job_id:priority=N or job_id:weight=W
            job, _, kv = spec.partition(":")
            k, _, v = kv.partition("=")
            if k not in ("priority", "weight"):
                raise SystemExit(f"bad update {spec!r}; use JOB:priority=N or JOB:weight=W")
            ups.append({"job_id": job, k: float(v) if k == "weight" else int(v)})
        session(a).post("/api/v1/job-queues/update", {"updates": ups})

    add(jb, "update-batch", job_update, (("updates",), {"nargs": "+"}))

    def task_config(a):
        print(json.dumps(session(a).get(f"/api/v1/tasks/{a.task_id}")["task"], indent=2, default=str))

    def task_kill(a):
        session(a).post(f"/api/v1/tasks/{a.task_id}/kill", {})

    add(tk, "config", task_config, "task_id")
    add(tk, "kill", task_kill, "task_id")


def register_template(tp: Any, session: Any) -> None:
    def describe(a):
        print(yaml.safe_dump(session(a).get(f"/api/v1/templates/{a.name}")["template"]["config"], sort_keys=False),
              end="")

    def remove(a):
        session(a).delete(f"/api/v1/templates/{a.name}")

    for verb, fn in (("describe", describe), ("remove", remove)):
        p = tp.add_parser(verb, aliases=["rm"] if verb == "remove" else [])
        p.add_argument("name")
        p.set_defaults(fn=fn)
