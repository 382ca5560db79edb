"""Fused AdamW for ``transformers.Trainer(optimizers=...)``.

HF's default ``torch.optim.AdamW`` runs a foreach multi-kernel update per step; on MI355X the
single-launch fused kernel (``csrc/optim.hip``) with bf16 master weights is the better choice.
The returned scheduler mirrors ``TrainingArguments.lr_scheduler_type`` via HF's own factory.
"""

from typing import Any, Tuple

import torch


def fused_optimizer(model: torch.nn.Module, args: Any, num_training_steps: int) -> Tuple[Any, Any]:
    from transformers import get_scheduler

    from determined_amd.ops import FusedAdamW

    decay, no_decay = [], []
    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        (no_decay if p.ndim < 2 or "norm" in n.lower() or n.endswith("bias") else decay).append(p)
    master = any(p.dtype == torch.bfloat16 for p in model.parameters())
    opt = FusedAdamW([{"params": decay, "weight_decay": args.weight_decay},
                      {"params": no_decay, "weight_decay": 0.0}],
                     lr=args.learning_rate, betas=(args.adam_beta1, args.adam_beta2), eps=args.adam_epsilon,
                     master_weights=master)
    sched = get_scheduler(args.lr_scheduler_type, opt, num_warmup_steps=args.get_warmup_steps(num_training_steps),
                          num_training_steps=num_training_steps)
    return opt, sched
