"""Web UI served by the master (reference: ``webui/react``, a React app over the REST API).

A dependency-free single-page app in ``master/webui/`` (no build step, no external assets -- the
cluster may have no egress), hash-routed over ``/api/v1``:

* Experiments: filterable list (name / label / state / project / archived) with bulk actions;
  experiment detail with overview (searcher-metric curves of every trial, best trial), trials table
  (one column per hyperparameter), hyperparameter visualisation (parallel coordinates coloured by
  the searcher metric + per-hyperparameter scatter plots), multi-trial metric comparison (any
  metric group / name), checkpoints, configuration and model-definition file tree;
* Trial detail: every metric group's curves, hyperparameters, checkpoints, live logs;
* Runs: the flat runs table (``POST /api/v1/runs``) with sorting and pagination;
* Projects: workspaces -> projects -> their experiments;
* Job queue: per resource pool, running jobs then the queue in scheduling order;
* Cluster: pool utilisation, agents with a per-slot map (busy / free / disabled) and enable /
  disable, 7-day allocation usage;
* Tasks (notebooks, shells, TensorBoards, commands) with logs; model registry with versions;
  Admin: users, groups, roles, webhooks, templates, master configuration.

The page long-polls ``/api/v1/stream`` and re-renders the current view when an entity it shows
changes.  With authentication enabled it asks for credentials and keeps the session token in
``localStorage``.
"""

import pathlib

ASSETS = pathlib.Path(__file__).resolve().parent / "webui"
_TYPES = {".html": "text/html; charset=utf-8", ".js": "application/javascript; charset=utf-8",
          ".css": "text/css; charset=utf-8"}


def asset(name: str) -> bytes:
    return (ASSETS / name).read_bytes()


def add_webui_routes(route, _Raw) -> None:
    def page(q, b):
        return _Raw(asset("index.html"), _TYPES[".html"])

    for path in ("/", "/det", "/det/", "/ui", "/ui/"):
        route("GET", path)(page)
    for name in ("app.js", "app.css"):
        route("GET", f"/ui/{name}")(lambda q, b, n=name: _Raw(asset(n), _TYPES[pathlib.Path(n).suffix]))
