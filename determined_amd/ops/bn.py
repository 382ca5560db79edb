"""Fused channels-last BatchNorm (+ residual add) (+ ReLU) backed by csrc/bn.hip.

``BatchNormAct2d`` is a drop-in ``nn.BatchNorm2d`` subclass (same parameters, buffers and
state-dict keys) whose forward takes an optional residual and applies ReLU in the same pass:
``y = relu(bn(x) + residual)``.  Training on a supported GPU tensor runs 2 kernels forward
(stats, apply) and 2 backward (reduce, apply) instead of stock PyTorch's 7 HBM passes; with a
residual the forward also writes a ReLU bit mask so the backward never re-reads the residual.
CPU tensors / unsupported shapes use the exact PyTorch composition.

``split_grad=True`` returns the output twice, ``(y, y_alias)``, for an output with two consumers
(a ResNet block output feeds the next block's conv1 and its shortcut).  Both handles share
storage, but autograd delivers their gradients separately and the backward kernels sum them
while reading (one HBM pass fewer than autograd's elementwise gradient accumulation).
"""

from typing import Optional

import torch
import torch.nn.functional as F
from torch import nn


def _sum_grads(a, b, mf):
    """(first, second) gradient for a split-output backward; either may be None."""
    if a is None:
        a, b = b, None
    if a is None:
        return None, None
    a = a.contiguous(memory_format=mf)
    return a, (None if b is None else b.contiguous(memory_format=mf))


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, residual, momentum, eps, relu, split=False,
                stats_part=None):
        from determined_amd import ops

        # residual + ReLU: the forward also emits a 1-bit-per-element ReLU mask, so the backward
        # reads M*C/8 bytes instead of the residual tensor in both of its passes.
        # stats_part: batch-statistic partials from the producing convolution (ops/conv.py)
        y, stats, mask = ops.ext().bn_act_fwd(x, weight, bias, running_mean, running_var, float(momentum),
                                              float(eps), residual, bool(relu), True, stats_part)
        masked = mask.numel() > 0
        ctx.save_for_backward(x, None if masked else residual, stats, weight, mask if masked else None)
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.set_materialize_grads(False)  # _sum_grads takes a missing half of a split pair as None
        if split:
            return y, y.detach()
        return y

    @staticmethod
    def backward(ctx, dy, dy2=None):
        from determined_amd import ops

        x, residual, stats, weight, mask = ctx.saved_tensors
        mf = torch.channels_last if x.dim() == 4 else torch.contiguous_format
        dy, dy2 = _sum_grads(dy, dy2, mf)
        if dy is None:
            return (None,) * 11
        if dy2 is not None and mask is None:  # unmasked path: plain sum
            dy, dy2 = dy + dy2, None
        dx, dg, db, dres = ops.ext().bn_act_bwd(dy, x, residual, stats, weight, bool(ctx.relu), bool(ctx.has_res),
                                                mask, dy2)
        return (dx, dg, db, None, None,
                dres if ctx.has_res else None, None, None, None, None, None)


class _BNReLUPoolFn(torch.autograd.Function):
    """``maxpool3x3s2p1(relu(bn(x)))`` for the ResNet stem (csrc/bn.hip ``bn_relu_maxpool``):
    the full-size activation is never written and the pooling backward is gathered inside the
    two BN-backward passes."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, split=False, stats_part=None):
        from determined_amd import ops

        y, idx, stats, xarg = ops.ext().bn_pool_fwd(x, weight, bias, running_mean, running_var, float(momentum),
                                                    float(eps), stats_part)
        ctx.save_for_backward(x, idx, stats, weight, xarg)
        ctx.mark_non_differentiable(idx, xarg)
        ctx.set_materialize_grads(False)
        if split:
            return y, y.detach()
        return y

    @staticmethod
    def backward(ctx, dy, dy2=None):
        from determined_amd import ops

        x, idx, stats, weight, xarg = ctx.saved_tensors
        dy, dy2 = _sum_grads(dy, dy2, torch.channels_last)
        if dy is None:
            return (None,) * 9
        dx, dg, db = ops.ext().bn_pool_bwd(dy, idx, x, stats, weight, dy2, xarg)
        return dx, dg, db, None, None, None, None, None, None


class _GlobalAvgPoolFn(torch.autograd.Function):
    """``x.mean((2, 3))`` of a channels-last activation; the backward writes the broadcast
    gradient straight into a channels-last tensor (csrc/bn.hip ``hw_broadcast_kernel``)."""

    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[2], x.shape[3])
        return x.mean((2, 3))

    @staticmethod
    def backward(ctx, g):
        from determined_amd import ops

        return ops.ext().global_avgpool_bwd(g.contiguous(), ctx.hw[0], ctx.hw[1])


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """``[N, C, H, W] -> [N, C]`` mean over H, W (``flatten(AdaptiveAvgPool2d(1)(x), 1)``)."""
    from determined_amd import ops

    if (x.is_cuda and x.dim() == 4 and x.shape[1] % 8 == 0 and x.dtype in (torch.bfloat16, torch.float32)
            and x.is_contiguous(memory_format=torch.channels_last) and ops.fusion_enabled("avgpool")):
        return _GlobalAvgPoolFn.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


def _torch_bn_act(bn: nn.BatchNorm2d, x, residual, relu, momentum):
    if bn.running_mean is not None and bn.running_mean.dtype != x.dtype:
        # low-precision activations with fp32 statistics: normalise in fp32
        w = bn.weight.float() if bn.weight is not None else None
        b = bn.bias.float() if bn.bias is not None else None
        y = F.batch_norm(x.float(), bn.running_mean, bn.running_var, w, b,
                         bn.training or not bn.track_running_stats, momentum, bn.eps).to(x.dtype)
    else:
        y = F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias,
                         bn.training or not bn.track_running_stats, momentum, bn.eps)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


class BatchNormAct2d(nn.BatchNorm2d):
    """``relu(BatchNorm2d(x) [+ residual])`` with the fused HIP kernels on channels-last input."""

    def __init__(self, num_features: int, act: bool = True, eps: float = 1e-5, momentum: Optional[float] = 0.1,
                 **kw) -> None:
        super().__init__(num_features, eps=eps, momentum=momentum, **kw)
        self.act = act

    # num_batches_tracked is counted on the host (one tiny device add per BN layer per step is
    # pure launch overhead: 53 launches/step in ResNet-50) and written into the buffer only when
    # a state dict is produced.
    _nbt_host: Optional[int] = None

    def _nbt(self) -> int:
        if self._nbt_host is None:
            self._nbt_host = int(self.num_batches_tracked.item()) if self.num_batches_tracked is not None else 0
        return self._nbt_host

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        if self.num_batches_tracked is not None and self._nbt_host is not None:
            self.num_batches_tracked.fill_(self._nbt_host)
        super()._save_to_state_dict(destination, prefix, keep_vars)

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)
        self._nbt_host = None

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, split_grad: bool = False,
                stats_part: Optional[torch.Tensor] = None):
        """``relu(bn(x) [+ residual])``; with ``split_grad`` a pair ``(y, y)`` of handles whose
        gradients are summed inside the fused backward (module docstring).  ``stats_part``: the
        [nb, 2, C] (sum, sum of squares) partials of ``x`` its producer already computed
        (``ops.conv.conv_bn_input``); training mode then skips the statistics pass."""
        y = self._forward(x, residual, split_grad, stats_part)
        return y if not split_grad or isinstance(y, tuple) else (y, y)

    def train_step_args(self):
        """(running_mean, running_var, momentum) for one training-mode forward; advances the host
        batch counter (shared by the fused entry points, ops/conv.py bn_act_conv)."""
        momentum = 0.0 if self.momentum is None else self.momentum
        if self.training and self.track_running_stats and self.num_batches_tracked is not None:
            self._nbt_host = self._nbt() + 1
            if self.momentum is None:
                momentum = 1.0 / float(self._nbt_host)
        rm = self.running_mean if self.track_running_stats else None
        rv = self.running_var if self.track_running_stats else None
        return rm, rv, momentum

    def kernel_path(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None) -> bool:
        """True when a training-mode forward of ``x`` runs on the fused HIP kernels."""
        if not (self.training and x.is_cuda and self.affine):
            return False
        from determined_amd import ops

        return bool(ops.ext().bn_supported(x)) and (residual is None or residual.stride() == x.stride())

    def _forward(self, x: torch.Tensor, residual: Optional[torch.Tensor], split: bool,
                 stats_part: Optional[torch.Tensor] = None):
        momentum = 0.0 if self.momentum is None else self.momentum
        if self.training and self.track_running_stats and self.num_batches_tracked is not None:
            self._nbt_host = self._nbt() + 1
            if self.momentum is None:
                momentum = 1.0 / float(self._nbt_host)
        if not x.is_cuda or not self.affine:
            return _torch_bn_act(self, x, residual, self.act, momentum)
        from determined_amd import ops

        e = ops.ext()
        if not e.bn_supported(x) or (residual is not None and residual.stride() != x.stride()):
            return _torch_bn_act(self, x, residual, self.act, momentum)
        if self.training or not self.track_running_stats:
            rm = self.running_mean if self.track_running_stats else None
            rv = self.running_var if self.track_running_stats else None
            # the in-kernel gradient sum needs the masked (residual + ReLU) backward
            split = split and residual is not None and self.act
            return _BNActFn.apply(x, self.weight, self.bias, rm, rv, residual, momentum, self.eps, self.act, split,
                                  stats_part)
        # eval: fold running statistics; one elementwise pass.
        scale = self.weight.float() * torch.rsqrt(self.running_var + self.eps)
        shift = self.bias.float() - self.running_mean * scale
        if torch.is_grad_enabled() and (x.requires_grad or self.weight.requires_grad):
            y = x * scale.view(1, -1, 1, 1).to(x.dtype) + shift.view(1, -1, 1, 1).to(x.dtype)
            if residual is not None:
                y = y + residual
            return F.relu(y) if self.act else y
        return e.bn_apply(x, scale, shift, residual, self.act)

    def forward_maxpool(self, x: torch.Tensor, pool: nn.MaxPool2d, split_grad: bool = False,
                        stats_part: Optional[torch.Tensor] = None):
        """``pool(self(x))`` with the fused stem kernels when ``pool`` is the ResNet 3x3/s2/p1
        max-pool, training mode and a supported channels-last GPU tensor; exact composition
        otherwise."""
        fusable = (self.act and self.affine and x.is_cuda and x.dim() == 4 and self.training and
                   self.track_running_stats and pool.kernel_size in (3, (3, 3)) and pool.stride in (2, (2, 2)) and
                   pool.padding in (1, (1, 1)) and pool.dilation in (1, (1, 1)) and not pool.ceil_mode and
                   not pool.return_indices)
        if fusable:
            from determined_amd import ops

            fusable = ops.ext().bn_supported(x) and x.is_contiguous(memory_format=torch.channels_last)
        if not fusable:
            y = pool(self(x))
            return (y, y) if split_grad else y
        momentum = 0.0 if self.momentum is None else self.momentum
        self._nbt_host = self._nbt() + 1
        if self.momentum is None:
            momentum = 1.0 / float(self._nbt_host)
        # stats_part: batch-statistic partials the producer of x already computed (ops/conv.py)
        return _BNReLUPoolFn.apply(x, self.weight, self.bias, self.running_mean, self.running_var, momentum, self.eps,
                                   split_grad, stats_part)

    def _apply(self, fn, recurse: bool = True):
        # Running statistics always stay fp32 (a bf16 running_var loses the update signal).
        super()._apply(fn, recurse)
        for name in ("running_mean", "running_var"):
            b = getattr(self, name, None)
            if b is not None and b.is_floating_point() and b.dtype != torch.float32:
                self._buffers[name] = b.float()
        return self

    def extra_repr(self) -> str:
        return super().extra_repr() + f", act={self.act}"
