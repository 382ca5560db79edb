"""MNIST PyTorchTrial (mirrors the reference tutorial examples/tutorials/mnist_pytorch).

Data is synthetic MNIST-shaped (1x28x28, 10 classes): no dataset downloads are possible here.
"""

from typing import Any, Dict

import torch
import torch.nn.functional as F

from determined_amd import pytorch
from determined_amd.datasets import mnist
from determined_amd.models.small import MNISTNet


class MNistTrial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        self.model = context.wrap_model(MNISTNet(
            n_filters1=context.get_hparam("n_filters1"), n_filters2=context.get_hparam("n_filters2"),
            dropout1=context.get_hparam("dropout1"), dropout2=context.get_hparam("dropout2")))
        self.optimizer = context.wrap_optimizer(torch.optim.Adadelta(self.model.parameters(),
                                                                     lr=context.get_hparam("learning_rate")))
        self.lr = context.wrap_lr_scheduler(torch.optim.lr_scheduler.StepLR(self.optimizer, 1, gamma=0.9),
                                            pytorch.LRScheduler.StepMode.STEP_EVERY_EPOCH)

    def build_training_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(mnist(True, self.context.get_data_config().get("train_size", 6000)),
                                  batch_size=self.context.get_per_slot_batch_size(), shuffle=True)

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        return pytorch.DataLoader(mnist(False, self.context.get_data_config().get("val_size", 1000)),
                                  batch_size=self.context.get_per_slot_batch_size())

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, torch.Tensor]:
        x, y = batch
        loss = F.cross_entropy(self.model(x), y)
        self.context.backward(loss)
        self.context.step_optimizer(self.optimizer)
        return {"loss": loss}

    def evaluate_batch(self, batch: Any, batch_idx: int) -> Dict[str, Any]:
        x, y = batch
        out = self.model(x)
        loss = F.cross_entropy(out, y)
        acc = (out.argmax(1) == y).float().mean()
        return {"validation_loss": loss, "accuracy": acc}


if __name__ == "__main__":
    # Local (off-cluster) training: `python model_def.py`
    import logging

    logging.basicConfig(level=logging.INFO)
    hparams = {"learning_rate": 1.0, "n_filters1": 32, "n_filters2": 64, "dropout1": 0.25, "dropout2": 0.5,
               "global_batch_size": 64}
    with pytorch.init(hparams=hparams) as ctx:
        trial = MNistTrial(ctx)
        pytorch.Trainer(trial, ctx).fit(max_length=pytorch.Epoch(1), validation_period=pytorch.Batch(50))
