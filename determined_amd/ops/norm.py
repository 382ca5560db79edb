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

    def forward(self, x: torch.Tensor) -> torch.Tensor:
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
