"""Checkpoint garbage collection task (reference: ``harness/determined/exec/gc_checkpoints.py``).

    python -m determined_amd.exec.gc_checkpoints --storage-config CFG.json \\
        --delete '["uuid", ...]' [--globs '["**/*.pt"]'] [--delete-tensorboards --experiment-id N] \\
        [--dry-run] [--report-to URL]

Deletes whole checkpoints (or only the files matching ``--globs``, leaving a partial checkpoint
whose remaining resources are reported) from the experiment's ``checkpoint_storage``.  The master
runs the same policy in-process for local clusters (``master/_core.py:gc_experiment_checkpoints``);
this entry point is what it schedules as a separate task when storage is not reachable from the
master process, and what an operator runs by hand.  JSON arguments may be given inline or as
``@path``.
"""

import argparse
import json
import logging
import os
import shutil
import sys
from typing import Any, Dict, List, Optional

from determined_amd import storage

logger = logging.getLogger("determined_amd.exec.gc_checkpoints")


def json_arg(val: str) -> Any:
    if val.startswith("@"):
        with open(val[1:]) as f:
            return json.load(f)
    if os.path.isfile(val):
        with open(val) as f:
            return json.load(f)
    return json.loads(val)


def delete_checkpoints(sm: storage.StorageManager, uuids: List[str], globs: Optional[List[str]],
                       dry_run: bool = False) -> Dict[str, Dict[str, int]]:
    """Returns ``{uuid: remaining resources}`` (empty dict = fully deleted)."""
    out: Dict[str, Dict[str, int]] = {}
    for u in uuids:
        if dry_run:
            logger.info("dry run: would delete %s (globs=%s)", u, globs)
            continue
        try:
            out[u] = sm.delete(u, globs)
            logger.info("deleted %s%s", u, f" ({len(out[u])} resources remain)" if out[u] else "")
        except Exception as e:  # one bad checkpoint must not stop the rest
            logger.warning("failed to delete %s: %s", u, e)
    return out


def delete_tensorboards(sm: storage.StorageManager, experiment_id: int, dry_run: bool = False) -> None:
    """Tensorboard event files live under ``<storage>/tensorboard/experiment/<id>``."""
    root = os.path.join(sm._base_path, "tensorboard", "experiment", str(experiment_id))
    if not os.path.isdir(root):
        return
    if dry_run:
        logger.info("dry run: would delete %s", root)
        return
    shutil.rmtree(root, ignore_errors=True)


def main(argv: List[str]) -> int:
    ap = argparse.ArgumentParser(description="checkpoint GC")
    ap.add_argument("--storage-config", type=json_arg, required=True)
    ap.add_argument("--delete", type=json_arg, default=[], help="JSON list of checkpoint uuids")
    ap.add_argument("--globs", type=json_arg, default=None, help="JSON list of globs (default: everything)")
    ap.add_argument("--experiment-id", type=int, default=None)
    ap.add_argument("--delete-tensorboards", action="store_true")
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("--report-to", default=None, help="master URL to PATCH remaining checkpoint resources")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(levelname)s: %(message)s")
    sm = storage.build(a.storage_config)
    uuids = a.delete["checkpoints"] if isinstance(a.delete, dict) else a.delete
    remaining = delete_checkpoints(sm, list(uuids), a.globs, a.dry_run)
    if a.delete_tensorboards:
        if a.experiment_id is None:
            ap.error("--delete-tensorboards needs --experiment-id")
        delete_tensorboards(sm, a.experiment_id, a.dry_run)
    if a.report_to and remaining:
        from determined_amd.common import api

        sess = api.Session(a.report_to)
        for u, res in remaining.items():
            sess.patch(f"/api/v1/checkpoints/{u}",
                       {"resources": res, "state": "PARTIALLY_DELETED" if res else "DELETED"})
    print(json.dumps({"deleted": sorted(remaining), "remaining": {u: r for u, r in remaining.items() if r}}))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
