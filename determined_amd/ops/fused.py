"""Fused LM-head loss and Linear bias gradient (``csrc/fused.hip``).

``lm_cross_entropy(logits, labels, vocab_size)`` computes the mean next-token cross-entropy
straight from the bf16 ``[B, T, Vp]`` LM-head output: no shifted slice, no fp32 copy of the
logits, one read forward, one read + one write backward (the gradient is written in place
over the logits, which are dead after the loss).  ``FusedLinear`` is ``nn.Linear`` whose
bias gradient is a single-pass column sum instead of a generic reduction.
"""

from typing import Any

import torch
import torch.nn.functional as F
from torch import nn


def _ext():
    from determined_amd import ops

    return ops.ext()


class _LMCrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, vocab_size: int, ignore_index: int, inplace_grad: bool):
        rows, lse = _ext().lm_ce_fwd(logits, labels, vocab_size, ignore_index)
        tgt = labels[:, 1:]
        n_valid = ((tgt != ignore_index) & (tgt >= 0) & (tgt < vocab_size)).sum().clamp_(min=1).float()
        ctx.save_for_backward(logits, labels, lse, n_valid)
        ctx.vocab_size, ctx.ignore_index, ctx.inplace = vocab_size, ignore_index, inplace_grad
        return rows.sum() / n_valid

    @staticmethod
    def backward(ctx, g):
        logits, labels, lse, n_valid = ctx.saved_tensors
        scale = (g.float() / n_valid).reshape(1)
        dlogits = logits if ctx.inplace else torch.empty_like(logits)
        _ext().lm_ce_bwd(logits, labels, lse, scale, ctx.vocab_size, ctx.ignore_index, dlogits)
        return dlogits, None, None, None, None


def lm_cross_entropy(logits: torch.Tensor, labels: torch.Tensor, vocab_size: int, ignore_index: int = -100,
                     inplace_grad: bool = True) -> torch.Tensor:
    """Mean cross-entropy of ``logits[:, t]`` against ``labels[:, t + 1]`` over the first
    ``vocab_size`` columns (padded columns excluded)."""
    if logits.is_cuda and logits.dtype == torch.bfloat16 and logits.is_contiguous() and logits.shape[-1] % 8 == 0:
        return _LMCrossEntropyFn.apply(logits, labels.contiguous(), int(vocab_size), int(ignore_index),
                                       bool(inplace_grad))
    V = logits.shape[-1]
    lg = logits[:, :-1, :vocab_size].reshape(-1, vocab_size)
    lg = lg.to(torch.promote_types(lg.dtype, torch.float32))
    del V
    return F.cross_entropy(lg, labels[:, 1:].reshape(-1), ignore_index=ignore_index)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = (dy2 @ weight).view(*dy.shape[:-1], weight.shape[1])
        if ctx.needs_input_grad[1]:
            dw = dy2.t() @ x.reshape(-1, x.shape[-1])
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = _ext().bias_grad(dy2, weight.dtype)
        return dx, dw, db


class _LinearGeluFn(torch.autograd.Function):
    """``gelu_tanh(x W^T + b)``: the GEMM (bias in the hipBLASLt epilogue) plus one GELU pass
    forward; backward fuses gelu' with the bias gradient (csrc/fused.hip)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        h = F.linear(x, weight, bias)
        ctx.save_for_backward(x, weight, h)
        return _ext().gelu_fwd(h)

    @staticmethod
    def backward(ctx, dg):
        x, weight, h = ctx.saved_tensors
        dh, db = _ext().gelu_bwd_bias(dg.contiguous(), h, weight.dtype)
        dh2 = dh.view(-1, dh.shape[-1])
        dx = (dh2 @ weight).view(*dh.shape[:-1], weight.shape[1]) if ctx.needs_input_grad[0] else None
        dw = dh2.t() @ x.reshape(-1, x.shape[-1]) if ctx.needs_input_grad[1] else None
        return dx, dw, (db if ctx.needs_input_grad[2] else None)


def linear_gelu(linear: nn.Linear, x: torch.Tensor) -> torch.Tensor:
    """``F.gelu(linear(x), approximate="tanh")`` with the fused HIP GELU kernels on bf16 GPU
    tensors; the plain composition elsewhere."""
    if x.is_cuda and x.dtype == torch.bfloat16 and linear.bias is not None and linear.out_features % 8 == 0 \
            and linear.weight.dtype == torch.bfloat16 and x.is_contiguous():
        return _LinearGeluFn.apply(x, linear.weight, linear.bias)
    return F.gelu(linear(x), approximate="tanh")


class FusedLinear(nn.Linear):
    """``nn.Linear`` with a single-pass bf16 bias-gradient kernel on the GPU."""

    def forward(self, x: torch.Tensor) -> Any:
        if x.is_cuda and x.dtype == torch.bfloat16 and self.bias is not None and self.out_features % 8 == 0 \
                and torch.is_grad_enabled():
            return _LinearFn.apply(x, self.weight, self.bias)
        return F.linear(x, self.weight, self.bias)
