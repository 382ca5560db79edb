"""Data loading helpers (reference: ``harness/determined/pytorch/_data.py``).

``DataLoader`` records the constructor arguments so the controller can rebuild it with a
rank-sharded, resumable (skip-N-batches), reproducibly shuffled batch sampler.
"""

import math
from typing import Any, Callable, Dict, Iterator, List, Optional, Sequence, Union

import numpy as np
import torch
from torch.utils.data import BatchSampler, Dataset, RandomSampler, SequentialSampler

from determined_amd.pytorch import samplers

TorchData = Union[Dict[str, torch.Tensor], Sequence[torch.Tensor], torch.Tensor]
_Data = Union[Dict[str, Any], Sequence[Any], Any]


class DataLoader:
    """Drop-in for ``torch.utils.data.DataLoader`` that the trial controller can shard/resume."""

    def __init__(self, dataset: Dataset, batch_size: Optional[int] = 1, shuffle: bool = False,
                 sampler: Optional[torch.utils.data.Sampler] = None, batch_sampler: Optional[BatchSampler] = None,
                 num_workers: int = 0, collate_fn: Optional[Callable] = None, pin_memory: bool = False,
                 drop_last: bool = False, timeout: float = 0, worker_init_fn: Optional[Callable] = None,
                 multiprocessing_context: Any = None, generator: Any = None, *, prefetch_factor: Optional[int] = None,
                 persistent_workers: bool = False) -> None:
        if batch_sampler is not None and (batch_size != 1 or shuffle or sampler is not None or drop_last):
            raise ValueError("batch_sampler is mutually exclusive with batch_size, shuffle, sampler, drop_last")
        if sampler is not None and shuffle:
            raise ValueError("sampler is mutually exclusive with shuffle")
        self.dataset = dataset
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.sampler = sampler
        self.batch_sampler = batch_sampler
        self.num_workers = num_workers
        self.collate_fn = collate_fn
        self.pin_memory = pin_memory
        self.drop_last = drop_last
        self.timeout = timeout
        self.worker_init_fn = worker_init_fn
        self.multiprocessing_context = multiprocessing_context
        self.generator = generator
        self.prefetch_factor = prefetch_factor
        self.persistent_workers = persistent_workers

    def _base_batch_sampler(self, seed: int) -> Any:
        if self.batch_sampler is not None:
            return self.batch_sampler
        sampler = self.sampler
        if sampler is None:
            sampler = SequentialSampler(self.dataset)  # type: ignore
            if self.shuffle:
                sampler = samplers.ReproducibleShuffleSampler(sampler, seed)
        return BatchSampler(sampler, self.batch_size or 1, self.drop_last)

    def get_data_loader(self, repeat: bool = False, skip: int = 0, num_replicas: int = 1, rank: int = 0,
                        seed: int = 0, shard_batches: bool = False) -> torch.utils.data.DataLoader:
        bs = self._base_batch_sampler(seed)
        if num_replicas > 1 and shard_batches:
            bs = samplers.DistributedSampler(bs, num_replicas, rank)  # batch i -> rank i % n, keeps the tail
        elif num_replicas > 1:
            bs = samplers.DistributedBatchSampler(bs, num_replicas, rank)
        if repeat:
            bs = samplers.RepeatBatchSampler(bs)
        if skip:
            bs = samplers.SkipBatchSampler(bs, skip)
        kw: Dict[str, Any] = {}
        if self.num_workers > 0:
            kw.update(prefetch_factor=self.prefetch_factor or 2, persistent_workers=self.persistent_workers,
                      multiprocessing_context=self.multiprocessing_context, timeout=self.timeout)
        return torch.utils.data.DataLoader(self.dataset, batch_sampler=bs, num_workers=self.num_workers,
                                           collate_fn=self.collate_fn, pin_memory=self.pin_memory,
                                           worker_init_fn=self.worker_init_fn, generator=self.generator, **kw)

    def __iter__(self) -> Iterator:
        return iter(self.get_data_loader())

    def __len__(self) -> int:
        return len(self._base_batch_sampler(0))


def dataset_repro_message(name: str, obj: Any) -> str:
    """The controller's error for a loader that is not a :class:`DataLoader` (reference
    ``pytorch._dataset_repro_warning``)."""
    return (f"{name}() returned a {type(obj).__name__}, not a determined_amd.pytorch.DataLoader, whose samplers "
            "make shuffling reproducible, resume at the right batch after a pause and shard the data across "
            "slots.  Return a determined_amd.pytorch.DataLoader, or call "
            "context.experimental.disable_dataset_reproducibility_checks() in the trial's __init__ to use any "
            "loader (reproducibility and sharding are then the loader's job).")


def adapt_batch_sampler(batch_sampler: Any, repeat: bool = False, skip: int = 0, num_replicas: int = 1,
                        rank: int = 0) -> Any:
    if num_replicas > 1:
        batch_sampler = samplers.DistributedBatchSampler(batch_sampler, num_replicas, rank)
    if repeat:
        batch_sampler = samplers.RepeatBatchSampler(batch_sampler)
    if skip:
        batch_sampler = samplers.SkipBatchSampler(batch_sampler, skip)
    return batch_sampler


def data_length(data: _Data) -> int:
    if isinstance(data, torch.Tensor):
        return len(data)
    if isinstance(data, dict):
        vals = list(data.values())
        return data_length(vals[0]) if vals else 0
    if isinstance(data, (list, tuple)):
        return data_length(data[0]) if data else 0
    if isinstance(data, np.ndarray):
        return len(data)
    raise TypeError(f"cannot determine batch length of {type(data)}; implement get_batch_length()")


def to_device(data: _Data, device: torch.device, warned_types: Optional[set] = None,
              non_blocking: bool = True) -> TorchData:
    if isinstance(data, torch.Tensor):
        return data.to(device, non_blocking=non_blocking)
    if isinstance(data, dict):
        return {k: to_device(v, device, warned_types, non_blocking) for k, v in data.items()}
    if isinstance(data, tuple) and hasattr(data, "_fields"):
        return type(data)(*(to_device(v, device, warned_types, non_blocking) for v in data))
    if isinstance(data, (list, tuple)):
        return type(data)(to_device(v, device, warned_types, non_blocking) for v in data)
    if isinstance(data, np.ndarray):
        return torch.from_numpy(data).to(device, non_blocking=non_blocking)
    return data


def _dataset_len(loader: Any) -> Optional[int]:
    try:
        return len(loader)
    except TypeError:
        return None


def epoch_length(loader: Any, num_replicas: int) -> int:
    n = _dataset_len(loader)
    if n is None:
        raise ValueError("training data loader must have a length to use epoch-based lengths")
    return max(n // num_replicas, 1) if num_replicas > 1 else n


def records_to_batches(records: int, global_batch_size: int) -> int:
    return math.ceil(records / global_batch_size)
