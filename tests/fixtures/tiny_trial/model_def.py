"""Tiny CPU PyTorchTrial used by the cluster e2e tests: optional first-attempt crash (restart
path), InvalidHP, and a learnable regression target so validation metrics move."""

import os

import torch
import torch.nn.functional as F

from determined_amd import core, pytorch


class _DS(torch.utils.data.Dataset):
    def __init__(self, n, seed):
        g = torch.Generator().manual_seed(seed)
        self.x = torch.randn(n, 8, generator=g)
        self.y = self.x @ torch.arange(1.0, 9.0) / 10

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return self.x[i], self.y[i]


class TinyTrial(pytorch.PyTorchTrial):
    def __init__(self, context):
        self.context = context
        hp = context.get_hparams()
        if hp.get("invalid", False):
            raise core.InvalidHP("invalid hyperparameter combination")
        self.model = context.wrap_model(torch.nn.Linear(8, 1))
        self.opt = context.wrap_optimizer(torch.optim.SGD(self.model.parameters(), lr=float(hp.get("lr", 0.1))))
        marker = hp.get("crash_marker")
        self.crash = bool(marker) and not os.path.exists(marker)
        if self.crash:
            open(marker, "w").close()

    def train_batch(self, batch, epoch_idx, batch_idx):
        if self.crash and batch_idx >= 2:
            raise RuntimeError("injected failure")
        x, y = batch
        loss = F.mse_loss(self.model(x).squeeze(-1), y)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        return {"loss": loss}

    def evaluate_batch(self, batch, batch_idx):
        x, y = batch
        return {"validation_loss": F.mse_loss(self.model(x).squeeze(-1), y)}

    def build_training_data_loader(self):
        return pytorch.DataLoader(_DS(256, 0), batch_size=self.context.get_per_slot_batch_size(), shuffle=True)

    def build_validation_data_loader(self):
        return pytorch.DataLoader(_DS(64, 1), batch_size=16)


class NoisyFailTrial(TinyTrial):
    """Prints a recognisable error line and fails every attempt (log-policy tests)."""

    def train_batch(self, batch, epoch_idx, batch_idx):
        if batch_idx >= 1:
            print("FATAL: ECC error detected on device", flush=True)
            raise RuntimeError("hardware fault (simulated)")
        return super().train_batch(batch, epoch_idx, batch_idx)
