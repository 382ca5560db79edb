"""``python -m determined_amd.master`` -- run the master service."""

import argparse
import logging
import os
import sys

import yaml

from determined_amd.master import Master, MasterServer


def main(argv=None) -> int:
    p = argparse.ArgumentParser("determined_amd.master")
    p.add_argument("--config-file", default=None,
                   help="master.yaml (keys: host, port, db, scheduler, fit, auth, resource_pools, resource_manager)")
    p.add_argument("--host", default=None)
    p.add_argument("--port", type=int, default=None)
    p.add_argument("--db", default=None, help="sqlite path (default ~/.local/share/determined_amd/master.db)")
    p.add_argument("--scheduler", choices=["priority", "fair_share", "round_robin"], default=None)
    p.add_argument("--fit", choices=["best", "worst"], default=None)
    p.add_argument("--no-preemption", action="store_true")
    p.add_argument("--auth-token", default=os.environ.get("DET_MASTER_TOKEN"))
    p.add_argument("--auth", choices=["none", "basic", "rbac"], default=None,
                   help="user authentication / authorization mode (default none: single-user node)")
    a = p.parse_args(argv)
    cfg = {}
    if a.config_file:
        with open(a.config_file) as f:
            cfg = yaml.safe_load(f) or {}
    host = a.host or cfg.get("host", "127.0.0.1")
    port = a.port or int(cfg.get("port", 8080))
    db = a.db or cfg.get("db") or os.path.expanduser("~/.local/share/determined_amd/master.db")
    if db != ":memory:":
        os.makedirs(os.path.dirname(db), exist_ok=True)
    rm = cfg.get("resource_manager") or {}  # reference master.yaml: resource_manager + resource_pools
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    m = Master(db_path=db, policy=a.scheduler or cfg.get("scheduler", "priority"), fit=a.fit or cfg.get("fit", "best"),
               preemption=not a.no_preemption and cfg.get("preemption", True),
               master_url=cfg.get("advertised_url", f"http://{host}:{port}"), auth_token=a.auth_token,
               auth=a.auth or cfg.get("auth", "none"), resource_pools=cfg.get("resource_pools"),
               default_compute_pool=rm.get("default_compute_resource_pool"),
               default_aux_pool=rm.get("default_aux_resource_pool"))
    srv = MasterServer(m, host, port)
    logging.getLogger("determined_amd.master").info(f"master listening on http://{host}:{srv.port}")
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        srv.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
