"""CheckpointContext (reference: ``harness/determined/core/_checkpoint.py``).

Checkpoints are directories identified by a random ``storage_id`` (uuid4) in checkpoint
storage, carrying a ``metadata.json``.  ``shard=True`` lets every rank contribute files (e.g.
ZeRO-partitioned optimizer states) to ONE checkpoint: rank 0 picks the id, every rank writes
its own files, metadata dicts are merged (conflicting keys are an error), and the chief reports
the merged resource list to the master.
"""

import contextlib
import enum
import json
import logging
import os
import pathlib
import shutil
import tempfile
import uuid
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple

from determined_amd import storage
from determined_amd.core._distributed import DistributedContext

logger = logging.getLogger("determined_amd.core")


class DownloadMode(enum.Enum):
    LocalWorkersShareDownload = "LOCAL_WORKERS_SHARE_DOWNLOAD"
    NoSharedDownload = "NO_SHARED_DOWNLOAD"


def merge_metadata(all_metadata: List[Dict[str, Any]]) -> Tuple[Dict[str, Any], Dict[str, List[int]]]:
    """Merge per-rank metadata; returns (merged, conflicts{key: [ranks]})."""
    merged: Dict[str, Any] = {}
    owner: Dict[str, int] = {}
    conflicts: Dict[str, List[int]] = {}

    def rec(dst: Dict[str, Any], src: Dict[str, Any], rank: int, prefix: str) -> None:
        for k, v in src.items():
            key = prefix + k
            if isinstance(v, dict) and isinstance(dst.get(k, {}), dict):
                rec(dst.setdefault(k, {}), v, rank, key + "/")
            elif k in dst and dst[k] != v:
                conflicts.setdefault(key, [owner.get(key, -1)]).append(rank)
            else:
                dst[k] = v
                owner.setdefault(key, rank)

    for r, md in enumerate(all_metadata):
        rec(merged, md or {}, r, "")
    return merged, conflicts


class CheckpointContext:
    def __init__(self, dist: DistributedContext, storage_manager: storage.StorageManager,
                 session: Any = None, task_id: Optional[str] = None, allocation_id: Optional[str] = None,
                 trial_id: Optional[int] = None, tensorboard_manager: Any = None) -> None:
        self._dist = dist
        self._storage_manager = storage_manager
        self._session = session
        self._task_id = task_id
        self._allocation_id = allocation_id
        self._trial_id = trial_id
        self._tensorboard_manager = tensorboard_manager

    # -- upload / download ------------------------------------------------------------------
    def upload(self, ckpt_dir: Optional[os.PathLike], metadata: Optional[Dict[str, Any]] = None, *,
               shard: bool = False, selector: Optional[Callable[[str], bool]] = None) -> str:
        if not shard:
            if self._dist.rank != 0:
                raise RuntimeError("cannot call .upload(shard=False) from non-chief worker")
            if ckpt_dir is None:
                raise RuntimeError("ckpt_dir is required for .upload(shard=False)")
            storage_id = str(uuid.uuid4())
        else:
            storage_id = self._dist.broadcast(str(uuid.uuid4()) if self._dist.rank == 0 else None)
        self._upload_as(storage_id, ckpt_dir, metadata, shard, selector)
        return storage_id

    def _upload_as(self, storage_id: str, ckpt_dir: Optional[os.PathLike], metadata: Optional[Dict[str, Any]],
                   shard: bool, selector: Optional[Callable[[str], bool]]) -> None:
        if not shard:
            assert ckpt_dir is not None
            self._write_metadata_file(ckpt_dir, metadata or {})
            resources = storage.list_directory(ckpt_dir)
            if selector is not None:
                resources = {k: v for k, v in resources.items() if selector(k) or k == "metadata.json"}
            self._storage_manager.upload(src=ckpt_dir, dst=storage_id, paths=sorted(resources))
            self._report_checkpoint(storage_id, resources, metadata or {})
            return
        resources: Dict[str, int] = {}
        self._dist.allgather_local(None)  # every local rank finished writing before anyone lists
        if ckpt_dir is not None:
            resources = storage.list_directory(ckpt_dir)
            if selector is not None:
                resources = {k: v for k, v in resources.items() if selector(k)}
            # local workers sharing one directory upload each file once (lowest local rank that has it)
            key = str(pathlib.Path(ckpt_dir).resolve())
            local = [(d, set(fs)) for d, fs in self._dist.allgather_local((key, sorted(resources)))]
            me = self._dist.local_rank
            resources = {f: n for f, n in resources.items()
                         if next(i for i, (d, fs) in enumerate(local) if d == key and f in fs) == me}
            if resources:
                self._storage_manager.upload(src=ckpt_dir, dst=storage_id, paths=sorted(resources))
        merged_md, merged_res = self._merge(metadata, resources)
        if self._dist.rank == 0:
            with tempfile.TemporaryDirectory() as td:
                self._write_metadata_file(td, merged_md)
                self._storage_manager.upload(src=td, dst=storage_id, paths=["metadata.json"])
            merged_res["metadata.json"] = len(json.dumps(merged_md))
            self._report_checkpoint(storage_id, merged_res, merged_md)

    def _merge(self, metadata: Optional[Dict[str, Any]], resources: Dict[str, int]):
        all_md = self._dist.allgather(metadata or {})
        all_res = self._dist.allgather(resources)
        merged, conflicts = merge_metadata(all_md)
        if conflicts:
            raise RuntimeError(f"sharded checkpoint metadata conflicts between ranks: {conflicts}")
        owners: Dict[str, int] = {}
        for r, res in enumerate(all_res):
            for k in res:
                if k.endswith("/"):
                    continue
                if k in owners:
                    raise RuntimeError(f"file {k} uploaded by ranks {owners[k]} and {r} in one sharded checkpoint")
                owners[k] = r
        out: Dict[str, int] = {}
        for res in all_res:
            out.update(res)
        return merged, out

    def download(self, storage_id: str, ckpt_dir: os.PathLike,
                 download_mode: DownloadMode = DownloadMode.LocalWorkersShareDownload,
                 selector: Optional[Callable[[str], bool]] = None) -> None:
        mode = DownloadMode(download_mode)
        if mode == DownloadMode.NoSharedDownload or self._dist.local_size == 1:
            self._storage_manager.download(src=storage_id, dst=ckpt_dir, selector=selector)
            return
        if self._dist.local_rank == 0:
            self._storage_manager.download(src=storage_id, dst=ckpt_dir, selector=selector)
        self._dist.broadcast_local(None)  # wait for the local chief

    def get_metadata(self, storage_id: str) -> Dict[str, Any]:
        with self._storage_manager.restore_path(storage_id) as p:
            mp = pathlib.Path(p) / "metadata.json"
            return json.loads(mp.read_text()) if mp.exists() else {}

    @contextlib.contextmanager
    def store_path(self, metadata: Optional[Dict[str, Any]] = None, *,
                   shard: bool = False) -> Iterator[Tuple[pathlib.Path, str]]:
        """Yield ``(path, storage_id)``; files written there become the checkpoint on exit."""
        if not shard and self._dist.rank != 0:
            raise RuntimeError("cannot call .store_path(shard=False) from non-chief worker")
        storage_id = str(uuid.uuid4()) if not shard else self._dist.broadcast(
            str(uuid.uuid4()) if self._dist.rank == 0 else None)
        if not getattr(self._storage_manager, "is_local", True):
            # object store: stage locally, then upload like .upload() (metadata, shard merge, report)
            with tempfile.TemporaryDirectory() as td:
                yield pathlib.Path(td), storage_id
                self._upload_as(storage_id, td, metadata, shard, None)
            return
        with self._storage_manager.store_path(storage_id) as path:
            yield pathlib.Path(path), storage_id
            resources = storage.list_directory(path)
        if not shard:
            self._write_metadata_file(path, metadata or {})
            resources["metadata.json"] = (pathlib.Path(path) / "metadata.json").stat().st_size
            self._report_checkpoint(storage_id, resources, metadata or {})
            return
        # shared filesystem: every rank wrote into the same directory
        merged_md, _ = self._merge(metadata, {})
        self._dist.broadcast(None)  # every rank finished writing
        if self._dist.rank == 0:
            self._write_metadata_file(path, merged_md)
            self._report_checkpoint(storage_id, storage.list_directory(path), merged_md)

    @contextlib.contextmanager
    def restore_path(self, storage_id: str,
                     download_mode: DownloadMode = DownloadMode.LocalWorkersShareDownload,
                     selector: Optional[Callable[[str], bool]] = None) -> Iterator[pathlib.Path]:
        try:
            with self._storage_manager.restore_path(storage_id, selector=selector) as p:
                yield pathlib.Path(p)
                return
        except NotImplementedError:
            pass
        with tempfile.TemporaryDirectory() as td:
            self.download(storage_id, td, download_mode, selector)
            yield pathlib.Path(td)

    def delete(self, storage_id: str, globs: Optional[List[str]] = None) -> None:
        self._storage_manager.delete(storage_id, globs)
        if self._session is not None:
            self._session.delete(f"/api/v1/checkpoints/{storage_id}")

    # -- internals ---------------------------------------------------------------------------
    @staticmethod
    def _write_metadata_file(ckpt_dir: os.PathLike, metadata: Dict[str, Any]) -> None:
        pathlib.Path(ckpt_dir).mkdir(parents=True, exist_ok=True)
        with open(pathlib.Path(ckpt_dir) / "metadata.json", "w") as f:
            json.dump(metadata, f, indent=2, sort_keys=True, default=str)

    def _report_checkpoint(self, storage_id: str, resources: Dict[str, int], metadata: Dict[str, Any]) -> None:
        if self._session is None:
            logger.info(f"checkpoint {storage_id} stored (off-cluster; not reported)")
            return
        self._session.post("/api/v1/checkpoints", {
            "uuid": storage_id,
            "task_id": self._task_id,
            "allocation_id": self._allocation_id,
            "trial_id": self._trial_id,
            "resources": resources,
            "metadata": metadata,
            "steps_completed": metadata.get("steps_completed"),
        })


class DummyCheckpointContext(CheckpointContext):
    def __init__(self, dist: DistributedContext, storage_manager: storage.StorageManager) -> None:
        super().__init__(dist, storage_manager)
