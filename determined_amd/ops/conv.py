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


class _Conv1x1Fn(torch.autograd.Function):
    """1x1 stride-1 convolution whose input gradient is one GEMM.  A channels-last activation is
    an [N*H*W, C] row-major matrix, so dX = dY @ W on hipBLASLt writes dX directly, where
    MIOpen's solvers zero-fill dX and then run a CK/igemm kernel.  The forward and the weight
    gradient stay on MIOpen (dW as dY^T @ X has K = N*H*W and is 2-15x slower as a GEMM; the
    forward as X @ W^T wins only on the channel-reducing 14x14/7x7 layers, ~0.15 ms/step total).
    Measured per shape at batch 512: profiles/conv1x1_gemm_ab_b512_1gpu.jsonl,
    profiles/conv1x1_fwd_gemm_ab_b512_1gpu.jsonl."""

    @staticmethod
    def forward(ctx, x, weight):
        ctx.save_for_backward(x, weight)
        return torch.nn.functional.conv2d(x, weight)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        n, cout, h, w = dy.shape
        cin = x.shape[1]
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
            dx = (dy2 @ weight.view(cout, cin)).view(n, h, w, cin).permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            dw = torch.ops.aten.convolution_backward(dy, x, weight, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                     [False, True, False])[1]
        return dx, dw


def conv1x1_gemm_wins(hw: int, cin: int, cout: int) -> bool:
    """Shapes where the GEMM input gradient beat MIOpen on MI355X at batch 512
    (profiles/conv1x1_gemm_ab_b512_1gpu.jsonl): every 14x14 / 7x7 layer, and the channel-reducing
    layers at 56x56 / 28x28."""
    return hw <= 14 or cin > cout


def conv1x1(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """``conv(x)`` for a bias-free 1x1 stride-1 convolution; bf16 channels-last inputs on the GPU
    take :class:`_Conv1x1Fn` where its GEMM input gradient is faster (``DAMD_DISABLE_FUSIONS=
    conv1x1_gemm`` turns it off)."""
    if (x.is_cuda and x.dtype == torch.bfloat16 and conv.weight.dtype == torch.bfloat16 and x.dim() == 4
            and conv.bias is None and conv.groups == 1 and conv.kernel_size == (1, 1) and conv.stride == (1, 1)
            and conv.padding == (0, 0) and conv.dilation == (1, 1) and x.requires_grad
            and x.is_contiguous(memory_format=torch.channels_last) and torch.is_grad_enabled()
            and conv1x1_gemm_wins(x.shape[2], conv.in_channels, conv.out_channels)):
        from determined_amd import ops

        if ops.fusion_enabled("conv1x1_gemm"):
            return _Conv1x1Fn.apply(x, conv.weight)
    return conv(x)
