"""Samplers for reproducible, resumable, distributed data loading
(reference: ``harness/determined/pytorch/samplers.py``)."""

from typing import Iterator, List

import torch
from torch.utils.data import BatchSampler, Sampler


class RepeatSampler(Sampler):
    """Repeats an underlying sampler forever."""

    def __init__(self, sampler: Sampler) -> None:
        self._sampler = sampler

    def __len__(self) -> int:
        return len(self._sampler)  # type: ignore

    def __iter__(self) -> Iterator:
        while True:
            yield from self._sampler


class RepeatBatchSampler(BatchSampler):
    def __init__(self, batch_sampler: BatchSampler) -> None:
        self._bs = batch_sampler

    def __len__(self) -> int:
        return len(self._bs)

    def __iter__(self) -> Iterator:
        while True:
            yield from self._bs


class DistributedSampler(Sampler):
    """Round-robin shard of an arbitrary sampler (not a dataset): rank r takes every
    num_workers-th index starting at r.  Unlike torch's DistributedSampler it does not pad,
    so validation sees every record exactly once."""

    def __init__(self, sampler: Sampler, num_workers: int, rank: int) -> None:
        self._sampler = sampler
        self._n = num_workers
        self._rank = rank

    def __len__(self) -> int:
        full = len(self._sampler)  # type: ignore
        return full // self._n + (1 if self._rank < full % self._n else 0)

    def __iter__(self) -> Iterator:
        for i, idx in enumerate(self._sampler):
            if i % self._n == self._rank:
                yield idx


class DistributedBatchSampler(BatchSampler):
    """Shards whole global batches: each global batch of ``batch_size * num_workers`` records
    is split into contiguous per-rank slices; incomplete trailing batches are dropped for
    training (every rank must take the same number of steps)."""

    def __init__(self, batch_sampler: BatchSampler, num_workers: int, rank: int) -> None:
        self._bs = batch_sampler
        self._n = num_workers
        self._rank = rank

    def __len__(self) -> int:
        return len(self._bs) // self._n

    def __iter__(self) -> Iterator:
        group: List = []
        for b in self._bs:
            group.append(b)
            if len(group) == self._n:
                yield group[self._rank]
                group = []


class SkipSampler(BatchSampler):
    def __init__(self, sampler: BatchSampler, skip: int) -> None:
        self._s = sampler
        self._skip = skip

    def __len__(self) -> int:
        return len(self._s)

    def __iter__(self) -> Iterator:
        it = iter(self._s)
        for _ in range(self._skip):
            next(it)
        yield from it


class SkipBatchSampler(SkipSampler):
    """Skip the first ``skip`` batches (resuming mid-epoch after a checkpoint restore)."""

    def __len__(self) -> int:
        return max(len(self._s) - self._skip, 0)


class ReproducibleShuffleSampler(Sampler):
    """Shuffle with a seeded generator; epoch e uses permutation(seed + e)."""

    def __init__(self, sampler: Sampler, seed: int) -> None:
        self._sampler = sampler
        self._seed = seed
        self._epoch = 0

    def __iter__(self) -> Iterator:
        idxs = list(self._sampler)
        g = torch.Generator()
        g.manual_seed(self._seed + self._epoch)
        self._epoch += 1
        for i in torch.randperm(len(idxs), generator=g).tolist():
            yield idxs[i]

    def __len__(self) -> int:
        return len(self._sampler)  # type: ignore


class ReproducibleShuffleBatchSampler(Sampler):
    def __init__(self, batch_sampler: BatchSampler, seed: int) -> None:
        self._bs = batch_sampler
        self._seed = seed
        self._epoch = 0

    def __iter__(self) -> Iterator:
        batches = list(self._bs)
        g = torch.Generator()
        g.manual_seed(self._seed + self._epoch)
        self._epoch += 1
        for i in torch.randperm(len(batches), generator=g).tolist():
            yield batches[i]

    def __len__(self) -> int:
        return len(self._bs)
