"""TensorBoard event files without TensorFlow (reference: ``harness/determined/tensorboard``).

``EventFileWriter`` writes the TFRecord-framed ``Event`` protobuf stream that TensorBoard reads
(scalar summaries), hand-encoding the few protobuf fields involved and the masked CRC-32C
framing.  ``TensorboardManager`` keeps a per-trial local log dir and mirrors it into checkpoint
storage under ``tensorboard/experiment/<exp>/trial/<trial>/`` on ``sync()``.
"""

import os
import pathlib
import shutil
import socket
import struct
import time
from typing import Any, Callable, Dict, Optional, Tuple

_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_TABLE.append(_c)


def crc32c(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc = _CRC_TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def _masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, wire: int) -> bytes:
    return _varint((num << 3) | wire)


def _bytes_field(num: int, payload: bytes) -> bytes:
    return _field(num, 2) + _varint(len(payload)) + payload


def encode_scalar_event(tag: str, value: float, step: int, wall_time: Optional[float] = None) -> bytes:
    v = _bytes_field(1, tag.encode()) + _field(2, 5) + struct.pack("<f", float(value))
    summary = _bytes_field(1, v)
    ev = _field(1, 1) + struct.pack("<d", wall_time or time.time()) + _field(2, 0) + _varint(int(step))
    return ev + _bytes_field(5, summary)


def encode_version_event() -> bytes:
    return _field(1, 1) + struct.pack("<d", time.time()) + _bytes_field(3, b"brain.Event:2")


def decode_records(path: str):
    """Yield raw record payloads (used by tests / tooling to read event files back)."""
    with open(path, "rb") as f:
        while True:
            hdr = f.read(12)
            if len(hdr) < 12:
                return
            (n,) = struct.unpack("<Q", hdr[:8])
            data = f.read(n)
            f.read(4)
            yield data


class EventFileWriter:
    def __init__(self, logdir: str, suffix: str = "") -> None:
        os.makedirs(logdir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}{suffix}"
        self.path = os.path.join(logdir, name)
        self._f = open(self.path, "ab")
        self._write(encode_version_event())

    def _write(self, data: bytes) -> None:
        hdr = struct.pack("<Q", len(data))
        self._f.write(hdr + struct.pack("<I", _masked_crc(hdr)) + data + struct.pack("<I", _masked_crc(data)))

    def add_scalar(self, tag: str, value: float, step: int) -> None:
        self._write(encode_scalar_event(tag, value, step))

    def flush(self) -> None:
        self._f.flush()

    def close(self) -> None:
        self._f.close()


class MetricWriter:
    """Writes reported training/validation metrics as scalars (numbers only)."""

    def __init__(self, logdir: str, rank: int = 0) -> None:
        self._w = EventFileWriter(logdir, suffix=f".rank{rank}")

    def write(self, group: str, step: int, metrics: Dict[str, Any]) -> None:
        prefix = "val_" if group == "validation" else ("" if group == "training" else group + "/")
        for k, v in metrics.items():
            if hasattr(v, "item") and getattr(v, "ndim", 0) == 0:
                v = v.item()
            if isinstance(v, (int, float)) and not isinstance(v, bool):
                self._w.add_scalar(prefix + k if not k.startswith("val_") else k, float(v), step)
        self._w.flush()

    def close(self) -> None:
        self._w.close()


class TensorboardManager:
    def __init__(self, base_path: pathlib.Path, storage_manager: Any, sync_path: str,
                 sync_on_close: bool = True) -> None:
        self.base_path = pathlib.Path(base_path)
        self.sync_on_close = sync_on_close  # TensorboardMode.AUTO on the chief
        self.base_path.mkdir(parents=True, exist_ok=True)
        self._sm = storage_manager
        self._sync_path = sync_path

    def sync(self, selector: Callable[[pathlib.Path], bool] = lambda _: True,
             mangler: Callable[[pathlib.Path, int], pathlib.Path] = lambda p, __: p, rank: int = 0) -> None:
        if self._sm is None:
            return
        if not getattr(self._sm, "is_local", True):  # object store: upload the (mangled) event files
            import tempfile

            with tempfile.TemporaryDirectory() as td:
                rels = []
                for p in self.base_path.rglob("*"):
                    if p.is_file() and selector(p):
                        rel = mangler(p.relative_to(self.base_path), rank)
                        (pathlib.Path(td) / rel).parent.mkdir(parents=True, exist_ok=True)
                        shutil.copy2(p, pathlib.Path(td) / rel)
                        rels.append(str(rel))
                if rels:
                    self._sm.upload(td, self._sync_path, paths=rels)
            return
        target = pathlib.Path(self._sm._base_path) / self._sync_path
        for p in self.base_path.rglob("*"):
            if p.is_file() and selector(p):
                rel = mangler(p.relative_to(self.base_path), rank)
                (target / rel).parent.mkdir(parents=True, exist_ok=True)
                shutil.copy2(p, target / rel)

    def close(self) -> None:
        if not self.sync_on_close:
            return
        try:
            self.sync()
        except Exception:
            pass


def build_manager(cfg: Dict[str, Any], info: Any, dist: Any, sync_on_close: bool = True,
                  write_metrics: bool = True) -> Tuple[TensorboardManager, Optional[MetricWriter]]:
    from determined_amd import storage

    sm = storage.build(cfg.get("tensorboard_storage") or cfg["checkpoint_storage"])
    base = pathlib.Path(os.environ.get("DET_TENSORBOARD_DIR", "/tmp/tensorboard")) / \
        f"exp-{info.trial.experiment_id}-trial-{info.trial.trial_id}"
    mgr = TensorboardManager(base, sm, f"tensorboard/experiment/{info.trial.experiment_id}/trial/{info.trial.trial_id}",
                             sync_on_close=sync_on_close)
    return mgr, (MetricWriter(str(base), dist.rank) if write_metrics else None)
