"""Flat runs, bulk experiment actions and the experiment detail reads the web UI / SDK use
(reference: ``master/internal/api_runs.go`` SearchRuns / MoveRuns, ``api_experiment.go``
ActivateExperiments .. DeleteExperiments (bulk, by ids or by filter), GetExperimentValidationHistory,
ExpMetricNames, GetModelDefTree / GetModelDefFile).

A "run" is a trial seen on its own (the reference's run = trial row + its experiment's project);
moving runs moves their experiments, which is only allowed when every trial of the experiment is
in the request (as the reference refuses to split a multi-trial search)."""

import base64
import io
import tarfile
from typing import Any, Callable, Dict, List, Optional


def add_runs_routes(route: Callable[[str, str], Callable], m: Any) -> None:
    from determined_amd.master._server import HTTPError, _guard_exp

    def _project_filter(b: Dict[str, Any]) -> Optional[Dict[str, str]]:
        pid = b.get("project_id")
        if pid is None:
            return None
        p = m.db.one("SELECT * FROM projects WHERE id=?", [int(pid)])
        if p is None:
            raise HTTPError(404, f"project {pid} not found")
        w = m.db.one("SELECT name FROM workspaces WHERE id=?", [p["workspace_id"]])
        return {"project": p["name"], "workspace": w["name"]}

    def _run_row(t: Dict[str, Any], e: Dict[str, Any]) -> Dict[str, Any]:
        cfg = e.get("config") or {}
        return {"id": t["id"], "experiment_id": t["experiment_id"], "state": t["state"], "hparams": t["hparams"],
                "start_time": t.get("start_time"), "end_time": t.get("end_time"),
                "searcher_metric": (cfg.get("searcher") or {}).get("metric"),
                "searcher_metric_value": t.get("searcher_metric"), "total_batches": t.get("total_batches") or 0,
                "checkpoint_uuid": t.get("latest_checkpoint"), "experiment_name": e.get("name"),
                "project": e.get("project"), "workspace": e.get("workspace"), "owner": e.get("owner"),
                "archived": bool(e.get("archived")), "external_run_id": t.get("external_id")}

    _SORT = {"id": "id", "start_time": "start_time", "end_time": "end_time", "state": "state",
             "searcher_metric_value": "searcher_metric", "total_batches": "total_batches"}

    @route("POST", "/api/v1/runs")
    def search_runs(q, b):
        """SearchRuns: trials of non-deleted experiments, filtered by project / experiment ids /
        states / archived, sorted (``sort: "field=asc|desc"``), paginated (offset / limit)."""
        where = ["e.state != 'DELETED'"]
        args: List[Any] = []
        pf = _project_filter(b)
        if pf is not None:
            where.append("e.project = ? AND e.workspace = ?")
            args += [pf["project"], pf["workspace"]]
        if b.get("experiment_ids"):
            ids = [int(i) for i in b["experiment_ids"]]
            where.append(f"t.experiment_id IN ({','.join('?' * len(ids))})")
            args += ids
        if b.get("states"):
            st = [str(s) for s in b["states"]]
            where.append(f"t.state IN ({','.join('?' * len(st))})")
            args += st
        if b.get("archived") is not None:
            where.append("e.archived = ?")
            args.append(1 if b["archived"] else 0)
        field, _, order = str(b.get("sort") or "id=asc").partition("=")
        col = _SORT.get(field)
        if col is None:
            raise HTTPError(400, f"cannot sort runs by {field!r} (one of {sorted(_SORT)})")
        direction = "DESC" if order.lower() == "desc" else "ASC"
        rows = m.db.all(f"SELECT t.* FROM trials t JOIN experiments e ON e.id = t.experiment_id WHERE "
                        f"{' AND '.join(where)} ORDER BY t.{col} {direction}, t.id ASC", args)
        total = len(rows)
        off = int(b.get("offset") or 0)
        lim = int(b.get("limit") or 0)
        rows = rows[off:off + lim] if lim > 0 else rows[off:]
        exps: Dict[int, Dict[str, Any]] = {}
        out = []
        for t in rows:
            eid = int(t["experiment_id"])
            if eid not in exps:
                exps[eid] = m.db.one("SELECT * FROM experiments WHERE id=?", [eid]) or {}
            out.append(_run_row(t, exps[eid]))
        return {"runs": out, "pagination": {"offset": off, "limit": lim, "total": total}}

    @route("POST", "/api/v1/runs/move")
    def move_runs(q, b):
        """MoveRuns: move the experiments of ``run_ids`` to ``destination_project_id``; an
        experiment moves only when all of its runs are listed."""
        from determined_amd.master._iam import AuthError

        ids = {int(i) for i in b.get("run_ids") or []}
        dest = b.get("destination_project_id")
        if dest is None:
            raise HTTPError(400, "destination_project_id is required")
        p = m.iam.project(int(dest))
        w = m.iam.workspace(p["workspace_id"])
        m.iam.require("edit", w["id"])
        if p["archived"] or w["archived"]:
            raise HTTPError(400, "destination project is archived")
        results = []
        by_exp: Dict[int, List[int]] = {}
        for rid in sorted(ids):
            t = m.db.one("SELECT experiment_id FROM trials WHERE id=?", [rid])
            if t is None:
                results.append({"id": rid, "error": "run not found"})
                continue
            by_exp.setdefault(int(t["experiment_id"]), []).append(rid)
        for eid, rids in sorted(by_exp.items()):
            all_ids = {int(r["id"]) for r in m.db.all("SELECT id FROM trials WHERE experiment_id=?", [eid])}
            if not all_ids <= set(rids):
                results += [{"id": r, "error": f"experiment {eid} has other runs: move them together"} for r in rids]
                continue
            try:
                _guard_exp(m, eid, "edit")
            except (HTTPError, AuthError) as e:
                results += [{"id": r, "error": str(e)} for r in rids]
                continue
            m.db.update("experiments", "id", eid, project=p["name"], workspace=w["name"])
            results += [{"id": r, "error": ""} for r in rids]
        return {"results": results}

    # ---------------------------------------------------------------- bulk experiment actions
    _ACTIONS = {"activate": lambda eid: m.activate_experiment(eid), "pause": lambda eid: m.pause_experiment(eid),
                "cancel": lambda eid: m.kill_experiment(eid), "kill": lambda eid: m.kill_experiment(eid),
                "archive": lambda eid: m.archive_experiment(eid, True),
                "unarchive": lambda eid: m.archive_experiment(eid, False),
                "delete": lambda eid: m.delete_experiment(eid)}

    def _bulk(action: str):
        def handler(q, b):
            """``{experiment_ids: [...]}`` or ``{filters: {project_id, states, archived}}``; one
            result per experiment (an error does not stop the others)."""
            ids = [int(i) for i in b.get("experiment_ids") or []]
            if not ids and b.get("filters") is not None:
                f = b["filters"]
                where, args = ["state != 'DELETED'"], []
                pf = _project_filter(f)
                if pf is not None:
                    where.append("project = ? AND workspace = ?")
                    args += [pf["project"], pf["workspace"]]
                if f.get("states"):
                    where.append(f"state IN ({','.join('?' * len(f['states']))})")
                    args += list(f["states"])
                if f.get("archived") is not None:
                    where.append("archived = ?")
                    args.append(1 if f["archived"] else 0)
                ids = [int(r["id"]) for r in m.db.all(f"SELECT id FROM experiments WHERE {' AND '.join(where)}", args)]
            results = []
            for eid in ids:
                try:
                    _guard_exp(m, eid, "edit")
                    _ACTIONS[action](eid)
                    results.append({"id": eid, "error": ""})
                except Exception as e:  # noqa: BLE001 -- reported per experiment
                    results.append({"id": eid, "error": str(e)})
            return {"results": results}
        return handler

    for action in _ACTIONS:
        route("POST", rf"/api/v1/experiments/bulk/{action}")(_bulk(action))

    # ---------------------------------------------------------------- experiment detail reads
    @route("GET", r"/api/v1/experiments/(\d+)/validation-history")
    def validation_history(q, b, eid):
        """The validations that improved the experiment's best searcher metric, in time order."""
        _guard_exp(m, eid, "view")
        cfg = (m.db.one("SELECT config FROM experiments WHERE id=?", [int(eid)]) or {}).get("config") or {}
        metric = (cfg.get("searcher") or {}).get("metric")
        smaller = bool((cfg.get("searcher") or {}).get("smaller_is_better", True))
        out, best = [], None
        if metric:
            rows = m.db.all("SELECT m.trial_id, m.steps_completed, m.metrics, m.ts FROM metrics m JOIN trials t ON "
                            "t.id = m.trial_id WHERE t.experiment_id=? AND m.group_name='validation' ORDER BY m.ts, "
                            "m.id", [int(eid)])
            for r in rows:
                v = (r["metrics"] or {}).get(metric)
                if not isinstance(v, (int, float)):
                    continue
                if best is None or (v < best if smaller else v > best):
                    best = v
                    out.append({"trial_id": r["trial_id"], "end_time": r["ts"], "searcher_metric": v,
                                "steps_completed": r["steps_completed"]})
        return {"validation_history": out}

    @route("GET", r"/api/v1/experiments/(\d+)/metric-names")
    def metric_names(q, b, eid):
        _guard_exp(m, eid, "view")
        names: Dict[str, set] = {}
        for r in m.db.all("SELECT m.group_name, m.metrics FROM metrics m JOIN trials t ON t.id = m.trial_id "
                          "WHERE t.experiment_id=?", [int(eid)]):
            names.setdefault(r["group_name"], set()).update((r["metrics"] or {}).keys())
        e = m.db.one("SELECT config FROM experiments WHERE id=?", [int(eid)])
        return {"metric_names": {g: sorted(v) for g, v in sorted(names.items())},
                "searcher_metric": ((e or {}).get("config") or {}).get("searcher", {}).get("metric")}

    def _model_tar(eid: str) -> tarfile.TarFile:
        _guard_exp(m, eid, "view")
        row = m.db.one("SELECT model_def FROM experiments WHERE id=?", [int(eid)])
        md = (row or {}).get("model_def")
        if not md:
            raise HTTPError(404, f"experiment {eid} has no model definition")
        if isinstance(md, str):
            md = base64.b64decode(md)
        return tarfile.open(fileobj=io.BytesIO(md))

    @route("GET", r"/api/v1/experiments/(\d+)/file_tree")
    def file_tree(q, b, eid):
        """GetModelDefTree: the model definition's files (path, size, is_dir)."""
        with _model_tar(eid) as tf:
            files = [{"path": ti.name, "is_dir": ti.isdir(), "content_length": ti.size} for ti in tf.getmembers()]
        return {"files": sorted(files, key=lambda f: f["path"])}

    @route("POST", r"/api/v1/experiments/(\d+)/file")
    def file_content(q, b, eid):
        """GetModelDefFile: one file of the model definition (base64)."""
        path = str(b.get("path") or "")
        with _model_tar(eid) as tf:
            try:
                ti = tf.getmember(path)
            except KeyError:
                raise HTTPError(404, f"{path} not in the model definition of experiment {eid}")
            if not ti.isfile():
                raise HTTPError(400, f"{path} is not a file")
            data = tf.extractfile(ti).read()  # type: ignore[union-attr]
        return {"file": base64.b64encode(data).decode()}
