"""Checkpoint storage managers (reference: ``harness/determined/common/storage``).

``shared_fs`` and ``directory`` are filesystem-backed (the MI355X node's local NVMe or a shared
mount).  ``s3`` / ``gcs`` / ``azure`` talk to the object stores' HTTP APIs directly
(``storage/cloud.py``: SigV4 / OAuth bearer / SharedKey signing) since the cloud SDKs are not part
of this image.
"""

import contextlib
import os
import pathlib
import shutil
from typing import Any, Callable, Dict, Iterator, List, Optional, Union

Selector = Optional[Callable[[str], bool]]


class StorageManager:
    """Abstract storage: ``upload(src_dir, storage_id)``, ``download(storage_id, dst_dir)``."""

    def __init__(self, base_path: str) -> None:
        self._base_path = str(base_path)

    def upload(self, src: Union[str, os.PathLike], dst: str, paths: Optional[List[str]] = None) -> None:
        raise NotImplementedError

    def download(self, src: str, dst: Union[str, os.PathLike], selector: Selector = None) -> None:
        raise NotImplementedError

    def delete(self, storage_id: str, globs: Optional[List[str]] = None) -> Dict[str, int]:
        raise NotImplementedError

    @contextlib.contextmanager
    def store_path(self, dst: str) -> Iterator[pathlib.Path]:
        raise NotImplementedError
        yield  # pragma: no cover

    @contextlib.contextmanager
    def restore_path(self, src: str, selector: Selector = None) -> Iterator[pathlib.Path]:
        raise NotImplementedError
        yield  # pragma: no cover

    def pre_store_path(self, dst: str) -> pathlib.Path:
        return pathlib.Path(self._base_path) / dst


def list_directory(root: Union[str, os.PathLike]) -> Dict[str, int]:
    """``{relative path: size}`` for every file/dir under root (dirs end with '/', size 0)."""
    root = pathlib.Path(root)
    out: Dict[str, int] = {}
    for dirpath, dirnames, filenames in os.walk(root):
        rel = pathlib.Path(dirpath).relative_to(root)
        for d in dirnames:
            out[str(rel / d) + "/" if str(rel) != "." else d + "/"] = 0
        for f in filenames:
            p = pathlib.Path(dirpath) / f
            key = str(rel / f) if str(rel) != "." else f
            out[key] = p.stat().st_size
    return out


class SharedFSStorageManager(StorageManager):
    """Checkpoints live in ``<base_path>/<storage_id>/`` on a (possibly shared) filesystem."""

    @classmethod
    def from_config(cls, cfg: Dict[str, Any], container_path: Optional[str] = None) -> "SharedFSStorageManager":
        base = container_path or cfg["host_path"]
        if cfg.get("storage_path"):
            sp = cfg["storage_path"]
            base = sp if os.path.isabs(sp) else os.path.join(base, sp)
        return cls(base)

    def upload(self, src, dst, paths=None) -> None:
        target = pathlib.Path(self._base_path) / dst
        src = pathlib.Path(src)
        if paths is None:
            shutil.copytree(src, target, dirs_exist_ok=True)
            return
        for rel in paths:
            s = src / rel
            t = target / rel
            if rel.endswith("/") or s.is_dir():
                t.mkdir(parents=True, exist_ok=True)
            else:
                t.parent.mkdir(parents=True, exist_ok=True)
                shutil.copy2(s, t)

    def download(self, src, dst, selector=None) -> None:
        source = pathlib.Path(self._base_path) / src
        if not source.exists():
            raise FileNotFoundError(f"checkpoint {src} not found in {self._base_path}")
        dst = pathlib.Path(dst)
        for rel, _ in list_directory(source).items():
            if rel.endswith("/"):
                (dst / rel).mkdir(parents=True, exist_ok=True)
                continue
            if selector is not None and not selector(rel):
                continue
            (dst / rel).parent.mkdir(parents=True, exist_ok=True)
            shutil.copy2(source / rel, dst / rel)

    def delete(self, storage_id: str, globs: Optional[List[str]] = None) -> Dict[str, int]:
        root = pathlib.Path(self._base_path) / storage_id
        if not root.exists():
            return {}
        if not globs or globs == ["**/*"]:
            shutil.rmtree(root, ignore_errors=True)
            return {}
        for g in globs:
            for p in root.glob(g):
                if p.is_file():
                    p.unlink()
        return list_directory(root)

    @contextlib.contextmanager
    def store_path(self, dst: str) -> Iterator[pathlib.Path]:
        p = pathlib.Path(self._base_path) / dst
        p.mkdir(parents=True, exist_ok=True)
        yield p

    @contextlib.contextmanager
    def restore_path(self, src: str, selector: Selector = None) -> Iterator[pathlib.Path]:
        p = pathlib.Path(self._base_path) / src
        if not p.exists():
            raise FileNotFoundError(f"checkpoint {src} not found in {self._base_path}")
        yield p


class DirectoryStorageManager(SharedFSStorageManager):
    """``type: directory`` -- a container path that is already mounted (no host_path)."""

    @classmethod
    def from_config(cls, cfg: Dict[str, Any], container_path: Optional[str] = None) -> "DirectoryStorageManager":
        return cls(cfg["container_path"])


def build(cfg: Dict[str, Any], container_path: Optional[str] = None) -> StorageManager:
    t = cfg.get("type")
    if t == "shared_fs":
        return SharedFSStorageManager.from_config(cfg, container_path)
    if t == "directory":
        return DirectoryStorageManager.from_config(cfg, container_path)
    if t == "s3":
        return S3StorageManager.from_config(cfg)
    if t == "gcs":
        return GCSStorageManager.from_config(cfg)
    if t == "azure":
        return AzureStorageManager.from_config(cfg)
    raise ValueError(f"unknown checkpoint_storage type {t!r}")


def from_string(s: str) -> StorageManager:
    """``s3://bucket/prefix``, ``gs://bucket/prefix`` or a local directory (Core API v2 / unmanaged)."""
    for scheme, cls in (("s3://", S3StorageManager), ("gs://", GCSStorageManager)):
        if s.startswith(scheme):
            bucket, _, prefix = s[len(scheme):].partition("/")
            return cls(bucket, prefix=prefix) if cls is GCSStorageManager else cls(bucket, prefix=prefix,
                                                                                   endpoint_url=os.environ.get(
                                                                                       "AWS_ENDPOINT_URL"))
    return SharedFSStorageManager(os.path.expanduser(s))


from determined_amd.storage.cloud import (  # noqa: E402
    AzureStorageManager,
    CloudStorageManager,
    GCSStorageManager,
    S3StorageManager,
)
