"""ResNet (v1.5: stride on the 3x3 conv) for the headline benchmark.

Same architecture/parameter count as torchvision's ``resnet50`` (25,557,032 params),
written for MI355X: the model is meant to run channels-last (NHWC) in bf16 so MIOpen
picks its NHWC implicit-GEMM (MFMA) convolutions and the 1x1 convolutions are plain
[N*H*W, Cin] x [Cin, Cout] GEMMs.  The reference only names the model (its
``examples/`` ResNet trials build torchvision's); torchvision is not in this image.
"""

from typing import List, Optional, Type

import torch
from torch import nn

from determined_amd.ops.bn import BatchNormAct2d, global_avg_pool
from determined_amd.ops import fusion_enabled
from determined_amd.ops.conv import LazyBNResidual, _materialise, bn_act_conv, conv_bn_input, stem_bn_pool


def conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 3, stride=stride, padding=1, bias=False)


def conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, 1, stride=stride, bias=False)


def _chainable(blk: nn.Module) -> bool:
    """Blocks whose forward is exactly the chained composition (no hooks on the block itself)."""
    return (isinstance(blk, (Bottleneck, BasicBlock)) and not blk._forward_hooks
            and not blk._forward_pre_hooks)


def _downsample(ds: nn.Module, x: torch.Tensor, lazy_bn: bool = False):
    """``ds(x)`` for the ``Sequential(conv1x1, BatchNormAct2d)`` shortcut, with the BN statistics
    from the conv epilogue.  ``lazy_bn``: return the BN as a :class:`LazyBNResidual` (its apply
    pass folds into the consumer's conv prologue; ``_chain_blocks``)."""
    if (isinstance(ds, nn.Sequential) and len(ds) == 2 and isinstance(ds[1], BatchNormAct2d)
            and not ds._forward_hooks and not ds._forward_pre_hooks and not ds[1]._forward_hooks
            and not ds[1]._forward_pre_hooks):
        y, part = conv_bn_input(ds[0], x)
        if lazy_bn and part is not None and not ds[1].act and ds[1].kernel_path(y):
            return LazyBNResidual(y, part, ds[1], ds[0])
        return ds[1](y, stats_part=part)
    return ds(x)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int = 1, downsample: Optional[nn.Module] = None) -> None:
        super().__init__()
        cout = width * self.expansion
        self.conv1 = conv1x1(cin, width)
        self.bn1 = BatchNormAct2d(width)
        self.conv2 = conv3x3(width, width, stride)
        self.bn2 = BatchNormAct2d(width)
        self.conv3 = conv1x1(width, cout)
        self.bn3 = BatchNormAct2d(cout)  # fused: relu(bn3(conv3) + identity)
        self.downsample = downsample

    def convs(self):
        return (self.conv1, self.conv2, self.conv3)

    def bns(self):
        return (self.bn1, self.bn2, self.bn3)

    def forward(self, x, split_grad: bool = False):
        """``x`` is a tensor or the ``(main, shortcut)`` pair of a split-gradient producer;
        ``split_grad`` makes this block's output such a pair (ops/bn.py).  Every conv hands its
        output's BatchNorm statistics to the BN from its epilogue (ops/conv.py conv_bn_input)."""
        xm, xs = x if isinstance(x, tuple) else (x, x)
        identity = xs if self.downsample is None else _downsample(self.downsample, xs)
        y, part = conv_bn_input(self.conv1, xm)
        out = self.bn1(y, stats_part=part)
        y, part = conv_bn_input(self.conv2, out)
        out = self.bn2(y, stats_part=part)
        y, part = conv_bn_input(self.conv3, out)
        return self.bn3(y, identity, split_grad=split_grad, stats_part=part)


def _chain_blocks(blocks, x, split: bool):
    """Run residual blocks back to back with every BN(+residual)+ReLU fused into the autograd node
    of the conv that consumes it (ops/conv.py bn_act_conv), including a block's output BN with the
    next block's first conv: the backward then fuses each BN's reduce pass into that conv's
    input-gradient epilogue.  Returns the last block's output.  Blocks expose ``convs``/``bns``
    (the main path, last BN takes the residual) and ``downsample``."""
    # lazy: the pre-BN tensor came out of a bn_act_conv node whose conv is stride 1 (1x1 / 3x3), which
    # can absorb this BN's backward apply pass into its input gradient (ops/conv.py _LazyBNGrad)
    pending = None  # (pre-BN output, its stats partials, residual, BN, lazy) of the previous block
    for i, blk in enumerate(blocks):
        convs, bns = blk.convs(), blk.bns()
        if pending is None:
            xm, xs = x if isinstance(x, tuple) else (x, x)
            y, part = conv_bn_input(convs[0], xm)
            lazy = False
        else:
            y_prev, p_prev, res_prev, bn_prev, lazy_prev = pending
            xs, y, part = bn_act_conv(bn_prev, y_prev, p_prev, res_prev, convs[0], lazy_grad=lazy_prev)
            lazy = _pro_conv(convs[0])
        identity = xs if blk.downsample is None else _downsample(blk.downsample, xs, lazy_bn=True)
        for bn, conv in zip(bns[:-1], convs[1:]):
            _, y, part = bn_act_conv(bn, y, part, None, conv, lazy_grad=lazy)
            lazy = _pro_conv(conv)
        pending = (y, part, identity, bns[-1], lazy)
    y, part, identity, bn, _ = pending
    return bn(y, _materialise(identity), stats_part=part)


def _pro_conv(conv: nn.Conv2d) -> bool:
    """Stride-1 1x1 and 3x3 (pad 1) convs: their input gradient can absorb the following BN's
    backward apply (1x1: generic-tile prologue; 3x3: halo prologue where it times faster --
    otherwise the parked gradient is materialised exactly as before)."""
    k = conv.kernel_size
    return conv.stride == (1, 1) and ((k == (1, 1) and conv.padding == (0, 0)) or (k == (3, 3) and conv.padding == (1, 1)))


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin: int, width: int, stride: int = 1, downsample: Optional[nn.Module] = None) -> None:
        super().__init__()
        self.conv1 = conv3x3(cin, width, stride)
        self.bn1 = BatchNormAct2d(width)
        self.conv2 = conv3x3(width, width)
        self.bn2 = BatchNormAct2d(width)
        self.downsample = downsample

    def convs(self):
        return (self.conv1, self.conv2)

    def bns(self):
        return (self.bn1, self.bn2)

    def forward(self, x, split_grad: bool = False):
        xm, xs = x if isinstance(x, tuple) else (x, x)
        identity = xs if self.downsample is None else _downsample(self.downsample, xs)
        y, part = conv_bn_input(self.conv1, xm)
        out = self.bn1(y, stats_part=part)
        y, part = conv_bn_input(self.conv2, out)
        return self.bn2(y, identity, split_grad=split_grad, stats_part=part)


class ResNet(nn.Module):
    def __init__(self, block: Type[nn.Module], layers: List[int], num_classes: int = 1000,
                 zero_init_residual: bool = True) -> None:
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = BatchNormAct2d(64)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):  # includes BatchNormAct2d
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def _make_layer(self, block, width: int, blocks: int, stride: int = 1) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != width * block.expansion:
            downsample = nn.Sequential(
                conv1x1(self.inplanes, width * block.expansion, stride),
                BatchNormAct2d(width * block.expansion, act=False),
            )
        mods = [block(self.inplanes, width, stride, downsample)]
        self.inplanes = width * block.expansion
        mods += [block(self.inplanes, width) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # Every activation between blocks feeds two consumers (next conv1 + shortcut): producers
        # hand out split-gradient pairs so the backward sums the two gradients inside the BN
        # kernels instead of in separate elementwise adds (ops/bn.py).
        split = fusion_enabled("split_grad")
        # stem conv + BN + ReLU + max-pool as one op: the conv's full-size output is never stored
        # (ops/conv.py stem_bn_pool; fallback: stem conv with BN statistics + bn1.forward_maxpool)
        x = stem_bn_pool(self.conv1, self.bn1, self.maxpool, x, split_grad=split)
        blocks = [b for layer in (self.layer1, self.layer2, self.layer3, self.layer4) for b in layer]
        if fusion_enabled("bn_conv") and all(_chainable(b) for b in blocks):
            x = _chain_blocks(blocks, x, split)
        else:
            for i, blk in enumerate(blocks):
                x = blk(x, split_grad=split and i + 1 < len(blocks))
        x = global_avg_pool(x)  # == flatten(self.avgpool(x), 1); fused channels-last backward
        return self.fc(x)


def resnet50(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, **kw)


def resnet18(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, **kw)
