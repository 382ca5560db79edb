"""Causal / full self-attention for the transformer models.

GPU (bf16, head dim 64 or 128): the hand-written MFMA flash-attention kernels in
``csrc/attention.hip`` (online softmax, no [T, T] matrix in HBM; backward recomputes P from the
saved log-sum-exp), with an optional key-padding mask (BERT batches) and in-kernel dropout on the
attention probabilities (a counter-based keep decision recomputed by the backward -- no mask is
stored).  ``qkv_attention`` takes the packed ``[B, T, 3, H, D]`` projection output directly and
writes dQ/dK/dV into ONE gradient buffer of that shape, so the backward needs no concatenation of
three gradients.

Anything else (CPU tensors, fp32, other head sizes) uses PyTorch's ``scaled_dot_product_attention``
-- on ROCm with the composable-kernel backend preferred.
"""

import math
from typing import Optional

import torch
import torch.nn.functional as F

_configured = False


def _configure() -> None:
    global _configured
    if _configured:
        return
    _configured = True
    if torch.version.hip is not None and hasattr(torch.backends.cuda, "preferred_rocm_fa_library"):
        try:
            torch.backends.cuda.preferred_rocm_fa_library("ck")
        except Exception:  # pragma: no cover - builds without CK FMHA
            pass


def _ext():
    from determined_amd import ops

    return ops.ext()


def _supported(*ts: torch.Tensor) -> bool:
    if not all(t.is_cuda for t in ts):
        return False
    e = _ext()
    return all(e.attn_supported(t) for t in ts)


def key_mask(valid: torch.Tensor) -> torch.Tensor:
    """The kernels' key-padding mask from a ``[B, T]`` validity mask (nonzero = attend): uint8
    rows padded with zeros to a multiple of 64 keys."""
    B, T = valid.shape
    km = torch.zeros(B, (T + 63) // 64 * 64, dtype=torch.uint8, device=valid.device)
    km[:, :T] = valid.to(torch.uint8) if valid.dtype != torch.bool else valid
    return km


def _seed(dropout_p: float, device: torch.device) -> Optional[torch.Tensor]:
    """The dropout stream of one call: a 1-element int64 GPU tensor the kernels read at run time (an async
    device RNG draw -- no host round trip, and a graph-captured step draws a fresh seed on every replay)."""
    return torch.randint(0, 2**31 - 1, (1,), device=device, dtype=torch.int64) if dropout_p > 0 else None


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal: bool, scale: float, km=None, dropout_p: float = 0.0, seed=None):
        o, lse = _ext().attn_fwd(q, k, v, causal, scale, km, dropout_p, 0, seed)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale, ctx.km, ctx.dropout_p, ctx.seed = causal, scale, km, dropout_p, seed
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        if not _ext().attn_supported(do):
            do = do.transpose(1, 2).contiguous().transpose(1, 2)
        B, H, T, D = q.shape
        g = torch.empty(3, B, T, H, D, dtype=q.dtype, device=q.device).permute(0, 1, 3, 2, 4)
        dq, dk, dv = g[0], g[1], g[2]
        _ext().attn_bwd(do, q, k, v, o, lse, dq, dk, dv, ctx.causal, ctx.scale, ctx.km, ctx.dropout_p, 0, ctx.seed)
        return dq, dk, dv, None, None, None, None, None


class _QKVFlashAttnFn(torch.autograd.Function):
    """Attention over a packed ``[B, T, 3, H, D]`` tensor; gradient is packed the same way."""

    @staticmethod
    def forward(ctx, qkv, causal: bool, scale: float, dropout_p: float = 0.0, seed=None):
        q, k, v = (qkv[:, :, i].permute(0, 2, 1, 3) for i in range(3))
        o, lse = _ext().attn_fwd(q, k, v, causal, scale, None, dropout_p, 0, seed)
        ctx.save_for_backward(qkv, o, lse)
        ctx.causal, ctx.scale, ctx.dropout_p, ctx.seed = causal, scale, dropout_p, seed
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        if not _ext().attn_supported(do):
            do = do.transpose(1, 2).contiguous().transpose(1, 2)
        q, k, v = (qkv[:, :, i].permute(0, 2, 1, 3) for i in range(3))
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = (dqkv[:, :, i].permute(0, 2, 1, 3) for i in range(3))
        _ext().attn_bwd(do, q, k, v, o, lse, dq, dk, dv, ctx.causal, ctx.scale, None, ctx.dropout_p, 0, ctx.seed)
        return dqkv, None, None, None, None


def flash_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True,
                    scale: Optional[float] = None, key_padding: Optional[torch.Tensor] = None,
                    dropout_p: float = 0.0) -> torch.Tensor:
    """Fused attention for ``[B, H, T, D]`` bf16 tensors on the GPU (raises if unsupported).
    ``key_padding``: a ``key_mask`` tensor (or a ``[B, T]`` validity mask); ``dropout_p``:
    attention-probability dropout (in-kernel)."""
    scale = 1.0 / math.sqrt(q.shape[-1]) if scale is None else scale
    if not _supported(q, k, v):
        raise ValueError("flash_attention needs bf16 GPU tensors [B,H,T,D] with D in {64,128} and a contiguous D")
    if key_padding is not None and (key_padding.dtype != torch.uint8 or key_padding.shape[1] % 64):
        key_padding = key_mask(key_padding)
    return _FlashAttnFn.apply(q, k, v, causal, float(scale), key_padding, float(dropout_p),
                              _seed(dropout_p, q.device))


def causal_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, dropout_p: float = 0.0) -> torch.Tensor:
    """``softmax(q k^T / sqrt(d) + causal_mask) v`` for ``[B, H, T, D]`` tensors."""
    if q.is_cuda and _supported(q, k, v):
        return _FlashAttnFn.apply(q, k, v, True, 1.0 / math.sqrt(q.shape[-1]), None, float(dropout_p),
                                  _seed(dropout_p, q.device))
    if q.is_cuda:
        _configure()
    return F.scaled_dot_product_attention(q, k, v, dropout_p=dropout_p, is_causal=True)


def qkv_attention(qkv: torch.Tensor, causal: bool = True, dropout_p: float = 0.0) -> torch.Tensor:
    """Attention over the packed projection ``qkv [B, T, 3, H, D]``; returns ``[B, H, T, D]``
    whose memory is ``[B, T, H, D]`` (merging heads afterwards is a free view)."""
    B, T, _, H, D = qkv.shape
    if qkv.is_cuda and qkv.is_contiguous() and qkv.dtype == torch.bfloat16 and D in (64, 128):
        return _QKVFlashAttnFn.apply(qkv, causal, 1.0 / math.sqrt(D), float(dropout_p), _seed(dropout_p, qkv.device))
    q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
    if qkv.is_cuda:
        _configure()
    return F.scaled_dot_product_attention(q, k, v, dropout_p=dropout_p, is_causal=causal)
