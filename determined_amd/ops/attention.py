"""Causal / full self-attention for the transformer models.

GPU (bf16, head dim 64 or 128, no attention-probability dropout): the hand-written MFMA
flash-attention kernels in ``csrc/attention.hip`` (online softmax, no [T, T] matrix in HBM;
backward recomputes P from the saved log-sum-exp).  ``qkv_attention`` takes the packed
``[B, T, 3, H, D]`` projection output directly and writes dQ/dK/dV into ONE gradient buffer of
that shape, so the backward needs no concatenation of three gradients.

Anything else (CPU tensors, fp32, other head sizes, dropout > 0) uses PyTorch's
``scaled_dot_product_attention`` -- on ROCm with the composable-kernel backend preferred.
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


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal: bool, scale: float):
        o, lse = _ext().attn_fwd(q, k, v, causal, scale)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        if not _ext().attn_supported(do):
            do = do.transpose(1, 2).contiguous().transpose(1, 2)
        B, H, T, D = q.shape
        g = torch.empty(3, B, T, H, D, dtype=q.dtype, device=q.device).permute(0, 1, 3, 2, 4)
        dq, dk, dv = g[0], g[1], g[2]
        _ext().attn_bwd(do, q, k, v, o, lse, dq, dk, dv, ctx.causal, ctx.scale)
        return dq, dk, dv, None, None


class _QKVFlashAttnFn(torch.autograd.Function):
    """Attention over a packed ``[B, T, 3, H, D]`` tensor; gradient is packed the same way."""

    @staticmethod
    def forward(ctx, qkv, causal: bool, scale: float):
        q, k, v = (qkv[:, :, i].permute(0, 2, 1, 3) for i in range(3))
        o, lse = _ext().attn_fwd(q, k, v, causal, scale)
        ctx.save_for_backward(qkv, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        if not _ext().attn_supported(do):
            do = do.transpose(1, 2).contiguous().transpose(1, 2)
        q, k, v = (qkv[:, :, i].permute(0, 2, 1, 3) for i in range(3))
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = (dqkv[:, :, i].permute(0, 2, 1, 3) for i in range(3))
        _ext().attn_bwd(do, q, k, v, o, lse, dq, dk, dv, ctx.causal, ctx.scale)
        return dqkv, None, None


def flash_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True,
                    scale: Optional[float] = None) -> torch.Tensor:
    """Fused attention for ``[B, H, T, D]`` bf16 tensors on the GPU (raises if unsupported)."""
    scale = 1.0 / math.sqrt(q.shape[-1]) if scale is None else scale
    if not _supported(q, k, v):
        raise ValueError("flash_attention needs bf16 GPU tensors [B,H,T,D] with D in {64,128} and a contiguous D")
    return _FlashAttnFn.apply(q, k, v, causal, float(scale))


def causal_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, dropout_p: float = 0.0) -> torch.Tensor:
    """``softmax(q k^T / sqrt(d) + causal_mask) v`` for ``[B, H, T, D]`` tensors."""
    if dropout_p == 0.0 and q.is_cuda and _supported(q, k, v):
        return _FlashAttnFn.apply(q, k, v, True, 1.0 / math.sqrt(q.shape[-1]))
    if q.is_cuda:
        _configure()
    return F.scaled_dot_product_attention(q, k, v, dropout_p=dropout_p, is_causal=True)


def qkv_attention(qkv: torch.Tensor, causal: bool = True, dropout_p: float = 0.0) -> torch.Tensor:
    """Attention over the packed projection ``qkv [B, T, 3, H, D]``; returns ``[B, H, T, D]``
    whose memory is ``[B, T, H, D]`` (merging heads afterwards is a free view)."""
    B, T, _, H, D = qkv.shape
    if dropout_p == 0.0 and qkv.is_cuda and qkv.is_contiguous() and qkv.dtype == torch.bfloat16 and D in (64, 128):
        return _QKVFlashAttnFn.apply(qkv, causal, 1.0 / math.sqrt(D))
    q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
    if qkv.is_cuda:
        _configure()
    return F.scaled_dot_product_attention(q, k, v, dropout_p=dropout_p, is_causal=causal)
