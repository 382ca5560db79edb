"""Synthetic datasets with the shapes of the reference examples (no network access for downloads).

Labels are a deterministic function of the inputs (argmax of fixed random projections), so the
models actually learn and validation metrics move -- enough to exercise searchers and early
stopping meaningfully.
"""

import torch
from torch.utils.data import Dataset


class SyntheticClassification(Dataset):
    def __init__(self, n: int, shape, num_classes: int, seed: int = 0, channels_last: bool = False,
                 dtype: torch.dtype = torch.float32, noise: float = 0.5) -> None:
        g = torch.Generator().manual_seed(seed)
        self.x = torch.randn(n, *shape, generator=g)
        proj = torch.randn(int(torch.tensor(shape).prod()), num_classes, generator=torch.Generator().manual_seed(1234))
        logits = self.x.reshape(n, -1) @ proj + noise * torch.randn(n, num_classes, generator=g)
        self.y = logits.argmax(1)
        if dtype != torch.float32:
            self.x = self.x.to(dtype)
        self.channels_last = channels_last

    def __len__(self) -> int:
        return len(self.y)

    def __getitem__(self, i: int):
        return self.x[i], self.y[i]


def mnist(train: bool = True, n: int = 0) -> SyntheticClassification:
    return SyntheticClassification(n or (6000 if train else 1000), (1, 28, 28), 10, seed=0 if train else 1)


def cifar10(train: bool = True, n: int = 0) -> SyntheticClassification:
    return SyntheticClassification(n or (5000 if train else 1000), (3, 32, 32), 10, seed=2 if train else 3)


class SyntheticImageNet(Dataset):
    """ImageNet-shaped (3x224x224, 1000 classes) samples generated on the fly."""

    def __init__(self, n: int = 12800, seed: int = 0) -> None:
        self.n = n
        self.seed = seed

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i: int):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        return torch.randn(3, 224, 224, generator=g), int(torch.randint(0, 1000, (1,), generator=g))


class SyntheticTokens(Dataset):
    """Language-model samples of ``seq_len`` token ids: arithmetic progressions
    ``(start + stride * j) mod V`` with a per-sample stride in [1, 16] and 10% random tokens.
    Learnable (the model has to infer the stride from context), so the loss falls; generated
    on the fly and vectorised, so it never bottlenecks a step."""

    def __init__(self, n: int, seq_len: int, vocab_size: int, seed: int = 0, noise: float = 0.1) -> None:
        self.n, self.seq_len, self.vocab, self.seed, self.noise = n, seq_len, vocab_size, seed, noise

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i: int) -> torch.Tensor:
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        start = torch.randint(0, self.vocab, (1,), generator=g)
        stride = torch.randint(1, 17, (1,), generator=g)
        toks = (start + stride * torch.arange(self.seq_len)) % self.vocab
        flip = torch.rand(self.seq_len, generator=g) < self.noise
        toks[flip] = torch.randint(0, self.vocab, (int(flip.sum()),), generator=g)
        return toks
