"""GPT-2 DeepSpeedTrial on the native ZeRO engine (BASELINE config: "GPT-2 345M DeepSpeedTrial
ZeRO-2 slots_per_trial=8").

The DeepSpeed config (``ds_config.json``: ZeRO-2, bf16, AdamW, WarmupDecayLR, clipping) is
overwritten from ``hparams.overwrite_deepspeed_args`` exactly like the reference's DeepSpeed
examples.  Data: synthetic token sequences (no dataset downloads are possible here).
"""

import os
from typing import Any, Dict, Iterator, Optional

import torch

from determined_amd import pytorch
from determined_amd.datasets import SyntheticTokens
from determined_amd.models.gpt2 import gpt2
from determined_amd.pytorch import deepspeed as det_ds

HERE = os.path.dirname(os.path.abspath(__file__))


def param_groups(model: torch.nn.Module, weight_decay: float):
    decay, no_decay = [], []
    for n, p in model.named_parameters():
        (no_decay if p.ndim < 2 or "ln" in n or n.endswith("bias") else decay).append(p)
    return [{"params": decay, "weight_decay": weight_decay}, {"params": no_decay, "weight_decay": 0.0}]


class GPT2Trial(det_ds.DeepSpeedTrial):
    def __init__(self, context: det_ds.DeepSpeedTrialContext) -> None:
        self.context = context
        hp = context.get_hparams()
        cfg_path = os.path.join(HERE, hp.get("deepspeed_config", "ds_config.json"))
        ds_config = det_ds.overwrite_deepspeed_config(cfg_path, hp.get("overwrite_deepspeed_args", {}))
        overrides = {k: hp[k] for k in ("n_layer", "n_embd", "n_head", "vocab_size", "n_positions") if k in hp}
        model = gpt2(hp.get("model", "gpt2-medium"), dropout=float(hp.get("dropout", 0.1)),
                     activation_checkpointing=bool(hp.get("activation_checkpointing", False)), **overrides)
        self.seq_len = int(hp.get("seq_len", model.config.n_positions))
        self.vocab = model.config.vocab_size
        wd = float(ds_config.get("optimizer", {}).get("params", {}).get("weight_decay", 0.0))
        engine, _, _, _ = det_ds.initialize(model=model, model_parameters=param_groups(model, wd), config=ds_config)
        self.model_engine = context.wrap_model_engine(engine)

    def train_batch(self, dataloader_iter: Optional[Iterator[Any]], epoch_idx: int, batch_idx: int
                    ) -> Dict[str, Any]:
        tokens = self.context.to_device(next(dataloader_iter))
        loss = self.model_engine(tokens, labels=tokens)
        self.model_engine.backward(loss)
        self.model_engine.step()
        return {"loss": loss}

    def evaluate_batch(self, dataloader_iter: Optional[Iterator[Any]], batch_idx: int) -> Dict[str, Any]:
        tokens = self.context.to_device(next(dataloader_iter))
        loss = self.model_engine(tokens, labels=tokens)
        return {"validation_loss": loss, "perplexity": torch.exp(loss.float())}

    def build_training_data_loader(self) -> pytorch.DataLoader:
        n = int(self.context.get_data_config().get("train_size", 100_000))
        return pytorch.DataLoader(SyntheticTokens(n, self.seq_len, self.vocab, seed=0),
                                  batch_size=self.context.train_micro_batch_size_per_gpu, shuffle=True,
                                  num_workers=int(self.context.get_data_config().get("workers", 2)),
                                  pin_memory=torch.cuda.is_available(), drop_last=True)

    def build_validation_data_loader(self) -> pytorch.DataLoader:
        n = int(self.context.get_data_config().get("val_size", 512))
        return pytorch.DataLoader(SyntheticTokens(n, self.seq_len, self.vocab, seed=1),
                                  batch_size=self.context.train_micro_batch_size_per_gpu, drop_last=True)
