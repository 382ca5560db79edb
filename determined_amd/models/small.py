"""Small reference models used by the tutorial configs (MNIST, CIFAR-10).

MNIST net mirrors the reference tutorial (examples/tutorials/mnist_pytorch/model_def.py):
two convs + dropout + two linears.  CIFAR-10 net mirrors the legacy cifar10_pytorch
example's small CNN.
"""

import torch
from torch import nn


class MNISTNet(nn.Module):
    def __init__(self, n_filters1: int = 32, n_filters2: int = 64, dropout1: float = 0.25,
                 dropout2: float = 0.5) -> None:
        super().__init__()
        self.net = nn.Sequential(
            nn.Conv2d(1, n_filters1, 3, 1),
            nn.ReLU(),
            nn.Conv2d(n_filters1, n_filters2, 3, 1),
            nn.ReLU(),
            nn.MaxPool2d(2),
            nn.Dropout(dropout1),
            nn.Flatten(),
            nn.Linear(144 * n_filters2, 128),
            nn.ReLU(),
            nn.Dropout(dropout2),
            nn.Linear(128, 10),
        )

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.net(x)


class CIFARNet(nn.Module):
    def __init__(self, layer1_dropout: float = 0.25, layer2_dropout: float = 0.25,
                 layer3_dropout: float = 0.5, width: int = 32) -> None:
        super().__init__()
        w = width
        self.net = nn.Sequential(
            nn.Conv2d(3, w, 3, padding=1), nn.ReLU(),
            nn.Conv2d(w, w, 3), nn.ReLU(),
            nn.MaxPool2d(2), nn.Dropout(layer1_dropout),
            nn.Conv2d(w, 2 * w, 3, padding=1), nn.ReLU(),
            nn.Conv2d(2 * w, 2 * w, 3), nn.ReLU(),
            nn.MaxPool2d(2), nn.Dropout(layer2_dropout),
            nn.Flatten(),
            nn.Linear(2 * w * 36, 512), nn.ReLU(),
            nn.Dropout(layer3_dropout),
            nn.Linear(512, 10),
        )

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.net(x)
