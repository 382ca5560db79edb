"""ResNet stem convolution (3 -> 64, 7x7, stride 2, pad 3) on the CDNA4 kernels of
csrc/conv_stem.hip: bf16 channels-last forward and weight gradient with the image rows staged
once per output row in LDS (channel dim padded 3 -> 4 so every im2col operand is one aligned
16-byte LDS read).  Anything else -- other shapes, fp32 inputs, an input that needs a gradient
-- runs the module's own convolution (MIOpen).
"""

import torch
from torch import nn


class _StemConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, want_stats):
        from determined_amd import ops

        ctx.save_for_backward(x, weight)
        y, part = ops.ext().stem_conv_fwd(x, weight, bool(want_stats))
        ctx.mark_non_differentiable(part)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart=None):
        from determined_amd import ops

        x, weight = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:  # images normally need no gradient
            dx = torch.nn.grad.conv2d_input(x.shape, weight.to(dy.dtype), dy, stride=2, padding=3)
        if ctx.needs_input_grad[1]:
            dw = ops.ext().stem_conv_wgrad(x, dy, weight)
        return dx, dw, None


def stem_fusable(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and conv.bias is None and conv.groups == 1
            and conv.in_channels == 3 and conv.out_channels == 64 and conv.kernel_size == (7, 7)
            and conv.stride == (2, 2) and conv.padding == (3, 3) and conv.dilation == (1, 1)
            and conv.padding_mode == "zeros" and conv.weight.dtype in (torch.bfloat16, torch.float32)
            and not x.requires_grad and x.is_contiguous(memory_format=torch.channels_last)):
        return False
    from determined_amd import ops

    return ops.fusion_enabled("stem_conv") and bool(ops.ext().stem_conv_supported(x, conv.weight))


def stem_conv2d(conv: nn.Conv2d, x: torch.Tensor, with_stats: bool = False):
    """``conv(x)`` for the ResNet stem convolution, on the HIP kernels when :func:`stem_fusable`.

    ``with_stats=True`` returns ``(y, part)`` where ``part`` holds the per-channel (sum, sum of
    squares) partials of ``y`` for the following BatchNorm (``BatchNormAct2d.forward_maxpool(...,
    stats_part=part)``) -- or ``None`` when the fallback convolution ran."""
    if stem_fusable(conv, x):
        from determined_amd import ops

        stats = with_stats and ops.fusion_enabled("stem_stats")
        y, part = _StemConvFn.apply(x, conv.weight, stats)
        if not with_stats:
            return y
        return y, (part if stats else None)
    y = conv(x)
    return (y, None) if with_stats else y
