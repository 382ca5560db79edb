"""BERT-base masked-LM pretraining with ``transformers.Trainer`` + ``DetCallback``
(BASELINE config: "BERT-base hf_trainer_api launcher slots_per_trial=4 bf16"; the reference's
HF examples live in ``examples/hf_trainer_api``).

Model: ``BertForMaskedLM`` from ``BertConfig()`` (bert-base-uncased shape, 110M params,
random init -- no checkpoint downloads are possible).  Data: synthetic token sequences with
BERT-style 15% masking (80% [MASK] / 10% random / 10% kept).  Optimizer: the fused
single-launch AdamW (``determined_amd.transformers.fused_optimizer``) unless
``--hf_optimizer`` is given.  Kernels: ``determined_amd.transformers.accelerate`` routes attention
(key-padding mask + in-kernel dropout) through csrc/attention.hip and residual + dropout + LayerNorm
through csrc/norm.hip unless ``--stock_kernels`` is given.

On-cluster:   python -m determined_amd.launch.torch_distributed python run_mlm.py [HF args]
Off-cluster:  python run_mlm.py --output_dir /tmp/bert --max_steps 50 ...
``hyperparameters.training_arguments`` in the experiment config override the HF arguments.
"""

import dataclasses
import logging
import os
import sys
from typing import Any, Dict, List, Optional

import torch
import transformers
from torch.utils.data import Dataset

from determined_amd import core
from determined_amd._info import get_cluster_info
from determined_amd.transformers import DetCallback, accelerate, fused_optimizer

logger = logging.getLogger("run_mlm")


class SyntheticMLM(Dataset):
    def __init__(self, n: int, seq_len: int, vocab: int, seed: int = 0, mask_id: int = 103) -> None:
        self.n, self.seq_len, self.vocab, self.seed, self.mask_id = n, seq_len, vocab, seed, mask_id

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i: int) -> Dict[str, torch.Tensor]:
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        start = torch.randint(1000, self.vocab, (1,), generator=g)
        stride = torch.randint(1, 9, (1,), generator=g)
        ids = 1000 + (start - 1000 + stride * torch.arange(self.seq_len)) % (self.vocab - 1000)
        ids[0] = 101  # [CLS]
        labels = torch.full_like(ids, -100)
        sel = torch.rand(self.seq_len, generator=g) < 0.15
        sel[0] = False
        labels[sel] = ids[sel]
        r = torch.rand(self.seq_len, generator=g)
        masked = ids.clone()
        masked[sel & (r < 0.8)] = self.mask_id
        rnd = sel & (r >= 0.8) & (r < 0.9)
        masked[rnd] = torch.randint(1000, self.vocab, (int(rnd.sum()),), generator=g)
        return {"input_ids": masked, "attention_mask": torch.ones_like(ids), "labels": labels}


@dataclasses.dataclass
class ModelArguments:
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    vocab_size: int = 30522
    seq_len: int = 128
    train_samples: int = 1_000_000
    eval_samples: int = 2048
    hf_optimizer: bool = False
    stock_kernels: bool = False
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    # bf16 parameters with fp32 master weights inside the fused AdamW (no per-step autocast weight casts)
    bf16_weights: bool = False


def dict2args(d: Dict[str, Any]) -> List[str]:
    out: List[str] = []
    for k, v in d.items():
        out += [f"--{k}", str(v)]
    return out


def parse(argv: List[str], hparams: Optional[Dict[str, Any]] = None):
    argv = list(argv) + dict2args((hparams or {}).get("training_arguments", {}))
    p = transformers.HfArgumentParser((ModelArguments, transformers.TrainingArguments))
    return p.parse_args_into_dataclasses(args=argv)


def build_model(m: ModelArguments, bf16: bool) -> torch.nn.Module:
    cfg = transformers.BertConfig(hidden_size=m.hidden_size, num_hidden_layers=m.num_hidden_layers,
                                  num_attention_heads=m.num_attention_heads, intermediate_size=m.intermediate_size,
                                  vocab_size=m.vocab_size, max_position_embeddings=max(512, m.seq_len),
                                  hidden_dropout_prob=m.hidden_dropout_prob,
                                  attention_probs_dropout_prob=m.attention_probs_dropout_prob,
                                  attn_implementation="sdpa")
    model = transformers.BertForMaskedLM(cfg)
    if not m.stock_kernels:
        accelerate(model)
    if m.bf16_weights:
        model = model.to(torch.bfloat16)
    return model


def main(core_context: Any, margs: ModelArguments, targs: transformers.TrainingArguments) -> Dict[str, Any]:
    model = build_model(margs, targs.bf16)
    train = SyntheticMLM(margs.train_samples, margs.seq_len, margs.vocab_size, seed=0)
    evald = SyntheticMLM(margs.eval_samples, margs.seq_len, margs.vocab_size, seed=1)
    det_cb = DetCallback(core_context, targs, user_data={"task": "mlm", "model": "bert-base"})
    optimizers = (None, None)
    if not margs.hf_optimizer:
        steps = targs.max_steps if targs.max_steps > 0 else \
            int(len(train) / (targs.per_device_train_batch_size * max(targs.world_size, 1)) * targs.num_train_epochs)
        optimizers = fused_optimizer(model, targs, steps)
    trainer = transformers.Trainer(model=model, args=targs, train_dataset=train, eval_dataset=evald,
                                   callbacks=[det_cb], optimizers=optimizers)
    result = trainer.train(resume_from_checkpoint=targs.resume_from_checkpoint)
    return {"train": result, "callback": det_cb}


if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO)
    info = get_cluster_info()
    hp = info.trial.hparams if info is not None and info.trial is not None else {}
    margs, targs = parse(sys.argv[1:], hp)
    distributed = core.DistributedContext.from_torch_distributed() if int(os.environ.get("WORLD_SIZE", "1")) > 1 \
        else None
    with core.init(distributed=distributed) as core_context:
        main(core_context, margs, targs)
