"""Tensor-parallel GPT-2 (Megatron layout) over ``parallel.tensor_parallel``.

Per block: fused QKV is column-parallel (heads split across the TP group, stride 3 so each
rank holds its heads' q, k and v), attention runs on the local heads with the MFMA flash
kernel, the output projection is row-parallel (one all-reduce); the MLP is column- then
row-parallel (one all-reduce).  Token embedding and the tied LM head are vocabulary-parallel
and the loss is ``vocab_parallel_cross_entropy`` -- the [tokens, vocab] logits are never
gathered.  Use with ``zero.initialize(..., mpu=tensor_parallel.get_mpu())`` so gradients are
averaged over the data-parallel group only.
"""

import math
from typing import Any, Dict, Optional

import torch
import torch.nn.functional as F
from torch import nn

from determined_amd.models.gpt2 import CONFIGS, GPT2Config
from determined_amd.ops.attention import qkv_attention
from determined_amd.ops.norm import FusedLayerNorm
from determined_amd.parallel import tensor_parallel as tp


def _normal(std: float):
    return lambda w: nn.init.normal_(w, mean=0.0, std=std)


class ParallelAttention(nn.Module):
    def __init__(self, cfg: GPT2Config) -> None:
        super().__init__()
        t = tp.get_tensor_model_parallel_world_size()
        if cfg.n_head % t:
            raise ValueError(f"n_head {cfg.n_head} not divisible by tensor-parallel size {t}")
        self.local_heads = cfg.n_head // t
        self.head_dim = cfg.n_embd // cfg.n_head
        self.c_attn = tp.ColumnParallelLinear(cfg.n_embd, 3 * cfg.n_embd, stride=3, init_method=_normal(0.02))
        self.c_proj = tp.RowParallelLinear(cfg.n_embd, cfg.n_embd,
                                           init_method=_normal(0.02 / math.sqrt(2 * cfg.n_layer)))
        self.resid_drop = nn.Dropout(cfg.dropout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        B, T, _ = x.shape
        qkv = self.c_attn(x).view(B, T, 3, self.local_heads, self.head_dim)
        y = qkv_attention(qkv, causal=True)
        y = y.transpose(1, 2).reshape(B, T, self.local_heads * self.head_dim)
        return self.resid_drop(self.c_proj(y))


class ParallelMLP(nn.Module):
    def __init__(self, cfg: GPT2Config) -> None:
        super().__init__()
        self.c_fc = tp.ColumnParallelLinear(cfg.n_embd, 4 * cfg.n_embd, init_method=_normal(0.02))
        self.c_proj = tp.RowParallelLinear(4 * cfg.n_embd, cfg.n_embd,
                                           init_method=_normal(0.02 / math.sqrt(2 * cfg.n_layer)))
        self.drop = nn.Dropout(cfg.dropout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.drop(self.c_proj(F.gelu(self.c_fc(x), approximate="tanh")))


class ParallelBlock(nn.Module):
    def __init__(self, cfg: GPT2Config) -> None:
        super().__init__()
        self.ln_1 = FusedLayerNorm(cfg.n_embd, eps=cfg.layer_norm_epsilon)
        self.attn = ParallelAttention(cfg)
        self.ln_2 = FusedLayerNorm(cfg.n_embd, eps=cfg.layer_norm_epsilon)
        self.mlp = ParallelMLP(cfg)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x + self.attn(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))


class GPT2TensorParallel(nn.Module):
    def __init__(self, cfg: GPT2Config) -> None:
        super().__init__()
        t = tp.get_tensor_model_parallel_world_size()
        self.config = cfg
        m = max(1, cfg.pad_vocab_to) * t
        self.padded_vocab = (cfg.vocab_size + m - 1) // m * m
        self.wte = tp.VocabParallelEmbedding(self.padded_vocab, cfg.n_embd, init_method=_normal(0.02))
        self.wpe = nn.Embedding(cfg.n_positions, cfg.n_embd)
        nn.init.normal_(self.wpe.weight, std=0.02)
        self.drop = nn.Dropout(cfg.dropout)
        self.h = nn.ModuleList([ParallelBlock(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = FusedLayerNorm(cfg.n_embd, eps=cfg.layer_norm_epsilon)

    def forward(self, input_ids: torch.Tensor, labels: Optional[torch.Tensor] = None) -> torch.Tensor:
        B, T = input_ids.shape
        x = self.drop(self.wte(input_ids) + self.wpe(torch.arange(T, device=input_ids.device)))
        for blk in self.h:
            x = blk(x)
        h = self.ln_f(x)
        logits = F.linear(tp.copy_to_tensor_model_parallel_region(h), self.wte.weight)  # [B, T, V/tp]
        if labels is None:
            return logits
        loss = tp.vocab_parallel_cross_entropy(logits[:, :-1], labels[:, 1:], vocab_start=self.wte.start,
                                               vocab_size=self.config.vocab_size)
        valid = (labels[:, 1:] != -100).sum().clamp(min=1)
        return loss.sum() / valid

    def load_from_dense(self, sd: Dict[str, Any]) -> None:
        """Load a ``GPT2LMHeadModel`` state dict (this rank keeps its shards)."""
        with torch.no_grad():
            wte = sd["wte.weight"]
            if wte.shape[0] < self.padded_vocab:
                wte = torch.cat([wte, wte.new_zeros(self.padded_vocab - wte.shape[0], wte.shape[1])])
            self.wte.load_full(wte[: self.padded_vocab])
            self.wpe.weight.copy_(sd["wpe.weight"])
            self.ln_f.weight.copy_(sd["ln_f.weight"])
            self.ln_f.bias.copy_(sd["ln_f.bias"])
            for i, blk in enumerate(self.h):
                p = f"h.{i}."
                for ln in ("ln_1", "ln_2"):
                    getattr(blk, ln).weight.copy_(sd[p + ln + ".weight"])
                    getattr(blk, ln).bias.copy_(sd[p + ln + ".bias"])
                blk.attn.c_attn.load_full(sd[p + "attn.c_attn.weight"], sd[p + "attn.c_attn.bias"])
                blk.attn.c_proj.load_full(sd[p + "attn.c_proj.weight"], sd[p + "attn.c_proj.bias"])
                blk.mlp.c_fc.load_full(sd[p + "mlp.c_fc.weight"], sd[p + "mlp.c_fc.bias"])
                blk.mlp.c_proj.load_full(sd[p + "mlp.c_proj.weight"], sd[p + "mlp.c_proj.bias"])


def gpt2_tp(name: str = "gpt2-medium", **overrides: Any) -> GPT2TensorParallel:
    kw = dict(CONFIGS[name])
    kw.update(overrides)
    return GPT2TensorParallel(GPT2Config(**kw))
