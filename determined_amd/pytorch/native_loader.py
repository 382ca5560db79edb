"""Native image-record loader: C++ worker threads -> pinned host ring -> async H2D on a side HIP
stream (the reference feeds trials through torch ``DataLoader`` worker processes,
``harness/determined/pytorch/_data.py``).

Why native: ResNet-50 at 9-10k images/s per MI355X needs ~1.5 GB/s of decoded bf16 pixels per
GPU and 8x that per node; Python worker processes pay pickling + shared-memory copies per batch.
Here ``_native.RecordLoader`` (``_native/loader.cpp``) mmaps a fixed-size record file, and its
threads crop/flip/normalise straight into pinned buffers owned by this module; each batch is
copied to the GPU with ``non_blocking=True`` on a dedicated stream and the compute stream waits
on an event, so the copy overlaps the previous step.

    write_record_file("train.rec", images_uint8_NHWC, labels)
    loader = NativeImageLoader("train.rec", batch_size=512, crop=(224, 224), device="cuda")
    for x, y in loader:          # x: [B, 3, 224, 224] bf16 channels-last view on the GPU
        ...
"""

import collections
import os
import struct
from typing import Any, Deque, Iterator, Optional, Sequence, Tuple

import numpy as np
import torch

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def write_record_file(path: str, images: np.ndarray, labels: Sequence[int]) -> None:
    """``images``: uint8 [N, H, W, C]; ``labels``: N ints.  Streams record by record."""
    images = np.asarray(images)
    if images.dtype != np.uint8 or images.ndim != 4:
        raise ValueError("images must be uint8 [N, H, W, C]")
    n, h, w, c = images.shape
    if len(labels) != n:
        raise ValueError("one label per image")
    with open(path, "wb") as f:
        f.write(b"DAMDREC1" + struct.pack("<qiiii", n, h, w, c, 0))
        for i in range(n):
            f.write(struct.pack("<i", int(labels[i])))
            f.write(np.ascontiguousarray(images[i]).tobytes())


def _native() -> Any:
    from determined_amd._native import load

    return load()


class NativeImageLoader:
    def __init__(self, path: str, batch_size: int, crop: Tuple[int, int] = (224, 224),
                 mean: Sequence[float] = IMAGENET_MEAN, std: Sequence[float] = IMAGENET_STD,
                 dtype: torch.dtype = torch.bfloat16, shuffle: bool = True, augment: bool = True,
                 drop_last: bool = True, seed: int = 0, rank: Optional[int] = None, world: Optional[int] = None,
                 workers: int = 8, prefetch: int = 4, device: Any = None) -> None:
        if dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("dtype must be bfloat16 or float32")
        if rank is None or world is None:
            if torch.distributed.is_available() and torch.distributed.is_initialized():
                rank, world = torch.distributed.get_rank(), torch.distributed.get_world_size()
            else:
                rank, world = 0, 1
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self._ld = _native().RecordLoader(os.fspath(path), int(batch_size), int(crop[0]), int(crop[1]),
                                          [float(m) for m in mean], [float(s) for s in std],
                                          dtype == torch.bfloat16, bool(shuffle), bool(augment), bool(drop_last),
                                          int(seed), int(rank), int(world), int(workers))
        _, _, c = self._ld.image_shape()
        pin = self.device.type == "cuda"
        self.batch_size = int(batch_size)
        self._data = [torch.empty((batch_size, crop[0], crop[1], c), dtype=dtype, pin_memory=pin)
                      for _ in range(max(2, prefetch))]
        self._labels = [torch.empty(batch_size, dtype=torch.int64, pin_memory=pin) for _ in self._data]
        self._ld.set_slots([t.data_ptr() for t in self._data], [t.data_ptr() for t in self._labels])
        self._stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self.epoch = 0

    def __len__(self) -> int:
        return int(self._ld.batches_per_epoch())

    @property
    def num_records(self) -> int:
        return int(self._ld.num_records())

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        ld = self._ld
        ld.start_epoch(self.epoch)
        inflight: Deque[Tuple[int, Any]] = collections.deque()  # (slot, copy-done event)
        try:
            while True:
                slot, n = ld.next()
                if slot < 0:
                    break
                x_h, y_h = self._data[slot][:n], self._labels[slot][:n]
                if self._stream is None:
                    x, y = x_h.clone(), y_h.clone()
                    ld.release(slot)
                else:
                    cur = torch.cuda.current_stream(self.device)
                    with torch.cuda.stream(self._stream):
                        x = x_h.to(self.device, non_blocking=True)
                        y = y_h.to(self.device, non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(self._stream)
                    cur.wait_event(ev)
                    x.record_stream(cur)
                    y.record_stream(cur)
                    inflight.append((slot, ev))
                    # hand slots back whose copies are done (keeps the ring full without a sync)
                    while inflight and (len(inflight) > 1 or inflight[0][1].query()):
                        s0, e0 = inflight.popleft()
                        e0.synchronize()
                        ld.release(s0)
                # NHWC storage presented as an NCHW channels-last tensor
                yield x.permute(0, 3, 1, 2), y
        finally:
            for s0, e0 in inflight:
                e0.synchronize()
                ld.release(s0)
            ld.stop()
        self.epoch += 1

    def close(self) -> None:
        self._ld.stop()
