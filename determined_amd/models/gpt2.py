"""GPT-2 (124M / 345M / 774M / 1.5B) decoder for the DeepSpeedTrial / ZeRO path.

BASELINE.json names "GPT-2 345M DeepSpeedTrial ZeRO-2 slots_per_trial=8"; the reference's
DeepSpeed example trains GPT-NeoX through DeepSpeed's engine (reference
``examples/deepspeed/gpt_neox``).  No HF weights can be downloaded here, so this is a
self-contained implementation of the GPT-2 architecture (pre-LN blocks, learned positions,
tied input/output embedding, GELU-tanh MLP) laid out for MI355X:

* bf16 weights and activations; LayerNorms are the wave-per-row fused HIP kernels
  (``ops.FusedLayerNorm``, ``csrc/norm.hip``), each fused with the residual add + dropout
  that precedes it (one kernel instead of dropout, add and LayerNorm);
* QKV / output / MLP projections are plain ``[B*T, d] x [d, n]`` GEMMs (hipBLASLt, MFMA);
* attention is the hand-written MFMA flash-attention kernel (``ops.attention.qkv_attention``,
  ``csrc/attention.hip``) on the packed QKV projection: no [T, T] score matrix in HBM and a
  packed QKV gradient;
* the vocabulary is padded to a multiple of 128 (50257 -> 50304) so the LM-head GEMM tiles
  evenly; padded logits are masked out of the loss;
* optional activation checkpointing per block.
"""

import dataclasses
import math
from typing import Any, Dict, Optional

import torch
import torch.nn.functional as F
from torch import nn
from torch.utils.checkpoint import checkpoint

from determined_amd.ops.attention import qkv_attention
from determined_amd.ops.fused import FusedLinear, linear_gelu, lm_cross_entropy
from determined_amd.ops.norm import FusedLayerNorm


@dataclasses.dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 1024
    n_layer: int = 24
    n_head: int = 16
    dropout: float = 0.1          # embedding / residual dropout
    attn_dropout: float = 0.0     # attention-probability dropout (off, as in GPT-NeoX configs)
    layer_norm_epsilon: float = 1e-5
    pad_vocab_to: int = 128
    activation_checkpointing: bool = False

    @property
    def padded_vocab(self) -> int:
        m = max(1, self.pad_vocab_to)
        return (self.vocab_size + m - 1) // m * m


CONFIGS: Dict[str, Dict[str, Any]] = {
    "gpt2": dict(n_embd=768, n_layer=12, n_head=12),            # 124M
    "gpt2-medium": dict(n_embd=1024, n_layer=24, n_head=16),    # 345M (355M w/ embeddings)
    "gpt2-large": dict(n_embd=1280, n_layer=36, n_head=20),     # 774M
    "gpt2-xl": dict(n_embd=1600, n_layer=48, n_head=25),        # 1.5B
    "gpt2-tiny": dict(n_embd=64, n_layer=2, n_head=4, vocab_size=512, n_positions=128),  # tests
}


class CausalSelfAttention(nn.Module):
    def __init__(self, cfg: GPT2Config) -> None:
        super().__init__()
        self.n_head = cfg.n_head
        self.c_attn = FusedLinear(cfg.n_embd, 3 * cfg.n_embd)
        self.c_proj = FusedLinear(cfg.n_embd, cfg.n_embd)
        self.attn_dropout = cfg.attn_dropout
        self.resid_drop = nn.Dropout(cfg.dropout)

    def forward(self, x: torch.Tensor, residual_dropout: bool = True) -> torch.Tensor:
        B, T, C = x.shape
        qkv = self.c_attn(x).view(B, T, 3, self.n_head, C // self.n_head)
        # fused MFMA flash attention on the packed projection; returns [B, H, T, D] laid out
        # as [B, T, H, D], so merging the heads below is a view
        y = qkv_attention(qkv, causal=True, dropout_p=self.attn_dropout if self.training else 0.0)
        y = y.transpose(1, 2).reshape(B, T, C)
        out = self.c_proj(y)
        return self.resid_drop(out) if residual_dropout else out


class MLP(nn.Module):
    def __init__(self, cfg: GPT2Config) -> None:
        super().__init__()
        self.c_fc = FusedLinear(cfg.n_embd, 4 * cfg.n_embd)
        self.c_proj = FusedLinear(4 * cfg.n_embd, cfg.n_embd)
        self.drop = nn.Dropout(cfg.dropout)

    def forward(self, x: torch.Tensor, residual_dropout: bool = True) -> torch.Tensor:
        out = self.c_proj(linear_gelu(self.c_fc, x))  # bias + GELU fused (ops/fused.py)
        return self.drop(out) if residual_dropout else out


class Block(nn.Module):
    def __init__(self, cfg: GPT2Config) -> None:
        super().__init__()
        self.ln_1 = FusedLayerNorm(cfg.n_embd, eps=cfg.layer_norm_epsilon)
        self.attn = CausalSelfAttention(cfg)
        self.ln_2 = FusedLayerNorm(cfg.n_embd, eps=cfg.layer_norm_epsilon)
        self.mlp = MLP(cfg)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x + self.attn(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))

    def forward_fused(self, x: torch.Tensor, h1: torch.Tensor, p: float):
        """Given the residual stream ``x`` and ``h1 = ln_1(x)``: returns ``(x', m)`` where
        ``x' = x + dropout(attn(h1))`` (fused with ``ln_2``) and ``m`` is the MLP branch whose
        residual add + dropout the caller fuses into the next LayerNorm."""
        a = self.attn(h1, residual_dropout=False)
        x, h2 = self.ln_2(x, branch=a, p=p)
        return x, self.mlp(h2, residual_dropout=False)


class GPT2LMHeadModel(nn.Module):
    def __init__(self, cfg: GPT2Config) -> None:
        super().__init__()
        self.config = cfg
        self.wte = nn.Embedding(cfg.padded_vocab, cfg.n_embd)
        self.wpe = nn.Embedding(cfg.n_positions, cfg.n_embd)
        self.drop = nn.Dropout(cfg.dropout)
        self.h = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = FusedLayerNorm(cfg.n_embd, eps=cfg.layer_norm_epsilon)
        self.apply(self._init)
        # GPT-2 scales the residual projections by 1/sqrt(2 * n_layer)
        for name, p in self.named_parameters():
            if name.endswith("c_proj.weight"):
                nn.init.normal_(p, mean=0.0, std=0.02 / math.sqrt(2 * cfg.n_layer))

    @staticmethod
    def _init(m: nn.Module) -> None:
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, mean=0.0, std=0.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, mean=0.0, std=0.02)

    def zero3_external_parameters(self):
        """ZeRO-3: the tied LM head reads ``wte.weight`` in this module's forward, and each MLP
        reads its ``c_fc`` parameters directly (fused bias + GELU, ops/fused.py linear_gelu)."""
        ext = [(self, self.wte.weight)]
        for blk in self.h:
            ext += [(blk.mlp, blk.mlp.c_fc.weight), (blk.mlp, blk.mlp.c_fc.bias)]
        return ext

    def num_parameters(self, exclude_embeddings: bool = False) -> int:
        n = sum(p.numel() for p in self.parameters())
        if exclude_embeddings:
            n -= self.wte.weight.numel() + self.wpe.weight.numel()
        return n

    def hidden_states(self, input_ids: torch.Tensor) -> torch.Tensor:
        B, T = input_ids.shape
        pos = torch.arange(T, device=input_ids.device)
        x = self.drop(self.wte(input_ids) + self.wpe(pos))
        ckpt = self.config.activation_checkpointing and self.training
        if not x.is_cuda:
            for blk in self.h:
                x = checkpoint(blk, x, use_reentrant=False) if ckpt else blk(x)
            return self.ln_f(x)
        # every residual add + dropout is fused into the following LayerNorm kernel
        # (ln_2 of the same block, ln_1 of the next, ln_f after the last)
        p = self.config.dropout if self.training else 0.0
        h = self.h[0].ln_1(x)
        for i, blk in enumerate(self.h):
            if ckpt:
                x, m = checkpoint(blk.forward_fused, x, h, p, use_reentrant=False)
            else:
                x, m = blk.forward_fused(x, h, p)
            nxt = self.h[i + 1].ln_1 if i + 1 < len(self.h) else self.ln_f
            x, h = nxt(x, branch=m, p=p)
        return h

    def forward(self, input_ids: torch.Tensor, labels: Optional[torch.Tensor] = None) -> Any:
        """Returns logits ``[B, T, vocab]`` or, with ``labels``, the mean next-token loss."""
        h = self.hidden_states(input_ids)
        logits = F.linear(h, self.wte.weight)  # tied LM head
        if labels is None:
            return logits[..., : self.config.vocab_size]
        return lm_loss(logits, labels, self.config.vocab_size)


def lm_loss(logits: torch.Tensor, labels: torch.Tensor, vocab_size: int) -> torch.Tensor:
    """Shifted next-token cross-entropy in fp32 (``-100`` labels ignored, padded vocab masked)."""
    return lm_cross_entropy(logits, labels, vocab_size, ignore_index=-100)


def gpt2(name: str = "gpt2-medium", **overrides: Any) -> GPT2LMHeadModel:
    kw = dict(CONFIGS[name])
    kw.update(overrides)
    return GPT2LMHeadModel(GPT2Config(**kw))
