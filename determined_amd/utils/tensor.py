"""Small tensor-layout helpers."""

import torch


def is_dense(t: torch.Tensor) -> bool:
    """True if ``t`` covers exactly ``numel`` contiguous elements in some dim order
    (e.g. contiguous or channels-last), i.e. it is non-overlapping and dense."""
    if t.numel() <= 1:
        return True
    dims = sorted(((st, sz) for st, sz in zip(t.stride(), t.shape) if sz != 1), key=lambda x: x[0])
    expected = 1
    for st, sz in dims:
        if st != expected:
            return False
        expected *= sz
    return True
