"""CIFAR-10 CNN PyTorchTrial for the adaptive-ASHA search config of BASELINE.json
("CIFAR-10 CNN adaptive_asha searcher, 32 trials max_concurrent_trials=8 across MI355X slots";
reference example: ``examples/legacy/computer_vision/cifar10_pytorch``).

Data is synthetic CIFAR-shaped (3x32x32, 10 classes, channels-last) -- no dataset downloads are
possible here.  Eight concurrent trials pack one MI355X node (8 slots, one trial per GPU); the
model is tiny, so every trial also keeps its batches on the GPU and steps with the fused
multi-tensor SGD kernel.
"""

from typing import Any, Dict

import torch
import torch.nn.functional as F

from determined_amd import ops, pytorch
from determined_amd.datasets import cifar10
from determined_amd.models.small import CIFARNet


class CIFARTrial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        self.model = context.wrap_model(CIFARNet(layer1_dropout=hp["layer1_dropout"],
                                                 layer2_dropout=hp["layer2_dropout"],
                                                 layer3_dropout=hp["layer3_dropout"]))
        params = self.model.parameters()
        if torch.cuda.is_available():
            opt = ops.FusedSGD(params, lr=hp["learning_rate"], momentum=hp["momentum"],
                               weight_decay=hp["weight_decay"], nesterov=True)
        else:
            opt = torch.optim.SGD(params, lr=hp["learning_rate"], momentum=hp["momentum"],
                                  weight_decay=hp["weight_decay"], nesterov=True)
        self.optimizer = context.wrap_optimizer(opt)

    def build_training_data_loader(self) -> pytorch.DataLoader:
        n = int(self.context.get_data_config().get("train_size", 50000))
        return pytorch.DataLoader(cifar10(True, n), batch_size=self.context.get_per_slot_batch_size(),
                                  shuffle=True, drop_last=True)

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        n = int(self.context.get_data_config().get("val_size", 10000))
        return pytorch.DataLoader(cifar10(False, n), batch_size=self.context.get_per_slot_batch_size())

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, torch.Tensor]:
        x, y = batch
        loss = F.cross_entropy(self.model(x), y)
        self.context.backward(loss)
        self.context.step_optimizer(self.optimizer)
        return {"loss": loss}

    def evaluate_batch(self, batch: Any, batch_idx: int) -> Dict[str, Any]:
        x, y = batch
        out = self.model(x)
        return {"validation_loss": F.cross_entropy(out, y), "accuracy": (out.argmax(1) == y).float().mean()}
