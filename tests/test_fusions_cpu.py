"""CPU behaviour of the model-level fusion entry points (the GPU paths are covered against fp32
references in tests/test_*_gpu.py): exact fallbacks, split-gradient pairs and the
DAMD_DISABLE_FUSIONS switches."""

import os
import subprocess
import sys

import torch
import torch.nn.functional as F

from determined_amd.models.resnet import resnet18, resnet50
from determined_amd.ops.bn import BatchNormAct2d, global_avg_pool
from determined_amd.ops.conv import stem_conv2d, stem_fusable
from determined_amd.ops.fused import linear_gelu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_split_grad_pair_on_cpu_sums_gradients():
    torch.manual_seed(0)
    bn = BatchNormAct2d(8)
    x = torch.randn(2, 8, 5, 5, requires_grad=True)
    r = torch.randn(2, 8, 5, 5)
    a, b = bn(x, r, split_grad=True)
    assert a is b  # CPU fallback hands out the same tensor twice; autograd sums the uses
    (a * 2 + b * 3).sum().backward()
    g1 = x.grad.clone()
    x.grad = None
    y = bn(x, r)
    (y * 5).sum().backward()
    torch.testing.assert_close(g1, x.grad)


def test_resnet_blocks_accept_pairs_and_tensors():
    torch.manual_seed(0)
    m = resnet50(num_classes=7)
    x = torch.randn(2, 3, 64, 64)
    out = m(x)
    h = m.bn1.forward_maxpool(m.conv1(x), m.maxpool)
    h = m.layer4(m.layer3(m.layer2(m.layer1(h))))
    ref = m.fc(torch.flatten(m.avgpool(h), 1))
    torch.testing.assert_close(out, ref)
    out18 = resnet18(num_classes=3)(x)
    assert out18.shape == (2, 3)


def test_stem_conv_and_pool_fallbacks_are_exact():
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
    x = torch.randn(2, 3, 32, 32)
    assert not stem_fusable(conv, x)
    torch.testing.assert_close(stem_conv2d(conv, x), conv(x))
    y, part = stem_conv2d(conv, x, with_stats=True)
    assert part is None
    torch.testing.assert_close(y, conv(x))
    z = torch.randn(2, 16, 5, 3)
    torch.testing.assert_close(global_avg_pool(z), torch.flatten(F.adaptive_avg_pool2d(z, 1), 1))


def test_linear_gelu_fallback_matches_composition():
    torch.manual_seed(0)
    lin = torch.nn.Linear(16, 32)
    x = torch.randn(4, 16)
    torch.testing.assert_close(linear_gelu(lin, x), F.gelu(lin(x), approximate="tanh"))


def test_disable_fusions_env_switch():
    code = ("import determined_amd.ops as o; "
            "print(o.fusion_enabled('split_grad'), o.fusion_enabled('stem_conv'), o.fusion_enabled('avgpool'))")
    env = dict(os.environ, PYTHONPATH=ROOT, DAMD_DISABLE_FUSIONS="split_grad, stem_conv")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    assert out.stdout.split() == ["False", "False", "True"]


def test_conv1x1_gemm_path_falls_back_on_cpu():
    from determined_amd.ops.conv import conv1x1, conv1x1_gemm_wins

    conv = torch.nn.Conv2d(32, 16, 1, bias=False)
    x = torch.randn(2, 32, 7, 7, requires_grad=True)
    torch.testing.assert_close(conv1x1(conv, x), conv(x))
    assert conv1x1_gemm_wins(14, 64, 256) and conv1x1_gemm_wins(56, 256, 64)
    assert not conv1x1_gemm_wins(56, 64, 256) and not conv1x1_gemm_wins(28, 128, 512)
