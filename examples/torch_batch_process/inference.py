"""Distributed batch inference with ``torch_batch_process`` (reference:
``examples/features/torch_batch_process_core_api_comparison/torch_batch_process_inference.py``).

Every slot runs a bf16 channels-last ResNet-18 over its shard of a (synthetic, CIFAR-shaped)
dataset, writes predictions per rank under the task's output directory, accumulates an
accuracy reducer that is all-gathered at the end, and checkpoints its progress every 20 batches
so a preempted / restarted task resumes where it stopped.

    det e create distributed.yaml .          # on a cluster (2 slots)
    python inference.py                      # locally (one worker)
"""

import json

import torch

from determined_amd import pytorch
from determined_amd.datasets import cifar10
from determined_amd.models.resnet import resnet18
from determined_amd.pytorch import experimental


class Accuracy(pytorch.MetricReducer):
    def __init__(self) -> None:
        self.reset()

    def reset(self) -> None:
        self.correct, self.total = 0, 0

    def update(self, correct: int, total: int) -> None:
        self.correct += correct
        self.total += total

    def per_slot_reduce(self):
        return self.correct, self.total

    def cross_slot_reduce(self, per_slot):
        c = sum(x[0] for x in per_slot)
        t = sum(x[1] for x in per_slot)
        return c / max(t, 1)


class Predictor(experimental.TorchBatchProcessor):
    def __init__(self, context: experimental.TorchBatchProcessorContext) -> None:
        self.context = context
        torch.manual_seed(0)
        use_gpu = context.device.type == "cuda"
        self.model = context.prepare_model_for_inference(resnet18(num_classes=10),
                                                         dtype=torch.bfloat16 if use_gpu else None,
                                                         channels_last=use_gpu)
        self.dtype = torch.bfloat16 if use_gpu else torch.float32
        self.acc = context.wrap_reducer(Accuracy(), name="accuracy")
        self.rows = []
        self.rank = context.get_distributed_rank()

    def process_batch(self, batch, batch_idx: int) -> None:
        x, y = self.context.to_device(batch)
        with torch.no_grad():
            pred = self.model(x.to(self.dtype)).argmax(1)
        self.acc.update(int((pred == y).sum()), int(y.numel()))
        self.rows += [{"batch": batch_idx, "pred": int(p)} for p in pred.tolist()]

    def on_checkpoint_start(self) -> None:
        # flush predictions accumulated since the last progress checkpoint
        if not self.rows:
            return
        with self.context.upload_path() as path:
            with open(path / f"predictions_rank{self.rank}.jsonl", "a") as f:
                for r in self.rows:
                    f.write(json.dumps(r) + "\n")
        self.rows = []

    def on_finish(self) -> None:
        self.on_checkpoint_start()


if __name__ == "__main__":
    experimental.torch_batch_process(Predictor, cifar10(False, 1024), batch_size=64, checkpoint_interval=20)
