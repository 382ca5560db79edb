"""LayerNorm / RMSNorm with the CDNA4 kernels of csrc/norm.hip (row-per-wave, register-resident rows).

GPU tensors always use the HIP kernels; CPU tensors use the PyTorch reference math.
"""

from typing import Optional, Sequence, Union

import torch
from torch import nn


def _ref_norm(x, weight, bias, eps, rms):
    xf = x.float()
    if rms:
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    else:
        mu = xf.mean(-1, keepdim=True)
        var = (xf - mu).pow(2).mean(-1, keepdim=True)
        y = (xf - mu) * torch.rsqrt(var + eps)
    y = y * weight.float()
    if bias is not None and not rms:
        y = y + bias.float()
    return y.to(x.dtype)


class _NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, rms):
        from determined_amd import ops

        xc = x.contiguous()
        y, mean, rstd = ops.ext().norm_fwd(xc, weight.contiguous(), bias, float(eps), bool(rms))
        ctx.save_for_backward(xc, weight, mean, rstd)
        ctx.rms = rms
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        from determined_amd import ops

        x, weight, mean, rstd = ctx.saved_tensors
        dx, dg, db = ops.ext().norm_bwd(dy.contiguous(), x, mean, rstd, weight.contiguous(), bool(ctx.rms))
        dg = dg.to(weight.dtype)
        db = db.to(weight.dtype) if ctx.has_bias else None
        return dx, dg, db, None, None


class _ResidNormFn(torch.autograd.Function):
    """``s = x + dropout(branch, p)``, ``y = LayerNorm(s)`` in one row-per-wave kernel
    (csrc/norm.hip RESID path); returns (s, y).  Backward: one kernel that adds the gradient
    arriving at ``s`` from its later use to the LayerNorm input-gradient and emits the branch
    gradient through the saved keep bits."""

    @staticmethod
    def forward(ctx, x, branch, weight, bias, eps, p, seed):
        from determined_amd import ops

        s, y, mean, rstd, mask = ops.ext().resid_norm_fwd(x.contiguous(), branch.contiguous(), weight.contiguous(),
                                                          bias, float(eps), float(p), 0, seed)
        ctx.save_for_backward(s, weight, mean, rstd, mask)
        ctx.p = float(p)
        ctx.has_bias = bias is not None
        ctx.mark_non_differentiable(mask)
        return s, y

    @staticmethod
    def backward(ctx, ds, dy):
        from determined_amd import ops

        s, weight, mean, rstd, mask = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(s)
        dx, dbranch, dg, db = ops.ext().resid_norm_bwd(dy.contiguous(), None if ds is None else ds.contiguous(), s,
                                                       mean, rstd, weight.contiguous(), mask, ctx.p, ctx.has_bias)
        return dx, dbranch, dg.to(weight.dtype), (db.to(weight.dtype) if ctx.has_bias else None), None, None, None


def residual_dropout_layer_norm(x: torch.Tensor, branch: torch.Tensor, norm: "FusedLayerNorm", p: float = 0.0,
                                training: bool = True):
    """``s = x + dropout(branch, p)``; returns ``(s, norm(s))``.  Fused on supported GPU tensors
    (H % 8 == 0, H <= 2048), exact PyTorch composition otherwise."""
    p = float(p) if training else 0.0
    if x.is_cuda:
        from determined_amd import ops

        e = ops.ext()
        if e.resid_norm_supported(x) and branch.dtype == x.dtype and branch.shape == x.shape:
            # device-side seed: no host round trip, a fresh draw on every replay of a captured graph
            seed = torch.randint(0, 2**31 - 1, (1,), device=x.device, dtype=torch.int64) if p > 0 else None
            return _ResidNormFn.apply(x, branch, norm.weight, norm.bias, norm.eps, p, seed)
    s = x + torch.nn.functional.dropout(branch, p, training=p > 0)
    return s, norm(s)


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor], eps: float = 1e-5):
    if not x.is_cuda:
        return _ref_norm(x, weight, bias, eps, False)
    return _NormFn.apply(x, weight, bias, eps, False)


def rms_norm(x: torch.Tensor, weight: torch.Tensor, eps: float = 1e-6):
    if not x.is_cuda:
        return _ref_norm(x, weight, None, eps, True)
    return _NormFn.apply(x, weight, None, eps, True)


class FusedLayerNorm(nn.Module):
    """Drop-in ``nn.LayerNorm`` (elementwise affine) over the last dimension."""

    def __init__(self, normalized_shape: Union[int, Sequence[int]], eps: float = 1e-5,
                 elementwise_affine: bool = True, bias: bool = True, device=None, dtype=None) -> None:
        super().__init__()
        if isinstance(normalized_shape, int):
            normalized_shape = (normalized_shape,)
        self.normalized_shape = tuple(normalized_shape)
        if len(self.normalized_shape) != 1:
            raise ValueError("FusedLayerNorm normalizes over the last dimension only")
        self.eps = eps
        self.elementwise_affine = elementwise_affine
        fk = {"device": device, "dtype": dtype}
        self.weight = nn.Parameter(torch.ones(self.normalized_shape, **fk), requires_grad=elementwise_affine)
        self.bias = nn.Parameter(torch.zeros(self.normalized_shape, **fk), requires_grad=elementwise_affine) \
            if bias else None

    def forward(self, x: torch.Tensor, branch: Optional[torch.Tensor] = None, p: float = 0.0):
        """``norm(x)``, or with ``branch``: ``(s, norm(s))`` for ``s = x + dropout(branch, p)``
        (residual add + dropout fused into the LayerNorm kernel)."""
        if branch is not None:
            return residual_dropout_layer_norm(x, branch, self, p, self.training)
        return layer_norm(x, self.weight, self.bias, self.eps)

    def extra_repr(self) -> str:
        return f"{self.normalized_shape}, eps={self.eps}"


class FusedRMSNorm(nn.Module):
    def __init__(self, hidden: int, eps: float = 1e-6, device=None, dtype=None) -> None:
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(hidden, device=device, dtype=dtype))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return rms_norm(x, self.weight, self.eps)
