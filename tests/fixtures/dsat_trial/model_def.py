"""Tiny DeepSpeedTrial for the autotuning e2e test; micro-batches above ``oom_above`` raise a
simulated HBM OOM (torch.OutOfMemoryError) the way a too-large candidate fails on a GPU."""

import os

import torch
from torch import nn

from determined_amd import pytorch
from determined_amd.pytorch import deepspeed as det_ds
from determined_amd.pytorch.dsat import get_ds_config_from_hparams

HERE = os.path.dirname(os.path.abspath(__file__))


class _Data(torch.utils.data.Dataset):
    def __len__(self):
        return 4096

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(i)
        x = torch.randn(16, generator=g)
        return x, x.sum(0, keepdim=True)


class TinyDSTrial(det_ds.DeepSpeedTrial):
    def __init__(self, context):
        self.context = context
        hp = context.get_hparams()
        self.oom_above = int(hp.get("oom_above", 1 << 30))
        cfg = get_ds_config_from_hparams(hp, HERE)
        torch.manual_seed(0)
        model = nn.Sequential(nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 1))
        engine, *_ = det_ds.initialize(model=model, config=cfg)
        self.engine = context.wrap_model_engine(engine)

    def train_batch(self, it, epoch_idx, batch_idx):
        x, y = next(it)
        if x.shape[0] > self.oom_above:
            raise torch.OutOfMemoryError(f"simulated: micro-batch {x.shape[0]} does not fit")
        loss = nn.functional.mse_loss(self.engine(x), y)
        self.engine.backward(loss)
        self.engine.step()
        return {"loss": loss}

    def evaluate_batch(self, it, batch_idx):
        x, y = next(it)
        return {"validation_loss": nn.functional.mse_loss(self.engine(x), y)}

    def build_training_data_loader(self):
        return pytorch.DataLoader(_Data(), batch_size=self.context.train_micro_batch_size_per_gpu, drop_last=True)

    def build_validation_data_loader(self):
        return pytorch.DataLoader(_Data(), batch_size=self.context.train_micro_batch_size_per_gpu, drop_last=True)
