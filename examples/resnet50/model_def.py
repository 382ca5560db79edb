"""ResNet-50 PyTorchTrial -- the headline benchmark model (BASELINE.json: "PyTorchTrial ResNet-50").

bf16 channels-last ResNet-50 with the fused NHWC BatchNorm+add+ReLU kernels, trained with the
fused multi-tensor SGD (momentum, no weight decay on BN/bias, fp32 master weights), linear
warm-up + cosine LR stepped per batch.  Data: synthetic ImageNet-shaped samples (no dataset
downloads are possible here).
"""

import math
from typing import Any, Dict

import torch
import torch.nn.functional as F

from determined_amd import pytorch
from determined_amd.datasets import SyntheticImageNet
from determined_amd.models.resnet import resnet50
from determined_amd.ops import FusedSGD


def param_groups(model: torch.nn.Module, weight_decay: float):
    decay, no_decay = [], []
    for p in model.parameters():
        (no_decay if p.ndim <= 1 else decay).append(p)
    return [{"params": decay, "weight_decay": weight_decay}, {"params": no_decay, "weight_decay": 0.0}]


class ResNet50Trial(pytorch.PyTorchTrial):
    def __init__(self, context: pytorch.PyTorchTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        self.dtype = torch.bfloat16 if hp.get("dtype", "bf16") == "bf16" else torch.float32
        model = resnet50(num_classes=int(hp.get("num_classes", 1000)))
        model = model.to(context.device).to(self.dtype).to(memory_format=torch.channels_last)
        self.model = context.wrap_model(model)
        gbs = context.get_global_batch_size()
        lr = float(hp.get("lr", 0.1)) * gbs / 256
        self.opt = context.wrap_optimizer(FusedSGD(param_groups(model, float(hp.get("weight_decay", 5e-5))), lr=lr,
                                                   momentum=float(hp.get("momentum", 0.9)),
                                                   nesterov=bool(hp.get("nesterov", False)),
                                                   master_weights=self.dtype == torch.bfloat16))
        warmup = int(hp.get("warmup_batches", 500))
        total = int(hp.get("total_batches", 50000))

        def schedule(step: int) -> float:
            if step < warmup:
                return (step + 1) / warmup
            return 0.5 * (1 + math.cos(math.pi * min(1.0, (step - warmup) / max(1, total - warmup))))

        self.sched = context.wrap_lr_scheduler(torch.optim.lr_scheduler.LambdaLR(self.opt, schedule),
                                               pytorch.LRScheduler.StepMode.STEP_EVERY_BATCH)

    def _prep(self, x: torch.Tensor) -> torch.Tensor:
        return x.to(self.context.device, self.dtype, non_blocking=True).contiguous(memory_format=torch.channels_last)

    def train_batch(self, batch: Any, epoch_idx: int, batch_idx: int) -> Dict[str, torch.Tensor]:
        x, y = batch
        logits = self.model(self._prep(x))
        loss = F.cross_entropy(logits.float(), y)
        self.context.backward(loss)
        self.context.step_optimizer(self.opt)
        return {"loss": loss}

    def evaluate_batch(self, batch: Any, batch_idx: int) -> Dict[str, Any]:
        x, y = batch
        logits = self.model(self._prep(x)).float()
        top5 = logits.topk(5, 1).indices
        return {"validation_loss": F.cross_entropy(logits, y),
                "accuracy": (top5[:, 0] == y).float().mean(),
                "top5_accuracy": (top5 == y[:, None]).any(1).float().mean()}

    def build_training_data_loader(self) -> pytorch.DataLoader:
        n = int(self.context.get_data_config().get("train_size", 128_000))
        return pytorch.DataLoader(SyntheticImageNet(n, seed=0), batch_size=self.context.get_per_slot_batch_size(),
                                  shuffle=True, num_workers=int(self.context.get_data_config().get("workers", 8)),
                                  pin_memory=True, drop_last=True)

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        n = int(self.context.get_data_config().get("val_size", 10_000))
        return pytorch.DataLoader(SyntheticImageNet(n, seed=1), batch_size=self.context.get_per_slot_batch_size(),
                                  num_workers=int(self.context.get_data_config().get("workers", 8)), pin_memory=True)
