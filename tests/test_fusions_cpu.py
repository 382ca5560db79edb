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
from determined_amd.ops.conv import stem_bn_pool, stem_conv2d, stem_fusable
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
    bn, pool = BatchNormAct2d(64), torch.nn.MaxPool2d(3, 2, 1)
    bn_ref = BatchNormAct2d(64)
    out = stem_bn_pool(conv, bn, pool, x)  # CPU: the unfused composition, running stats updated once
    torch.testing.assert_close(out, pool(bn_ref(conv(x))))
    torch.testing.assert_close(bn.running_mean, bn_ref.running_mean)


def test_linear_gelu_fallback_matches_composition():
    torch.manual_seed(0)
    lin = torch.nn.Linear(16, 32)
    x = torch.randn(4, 16)
    torch.testing.assert_close(linear_gelu(lin, x), F.gelu(lin(x), approximate="tanh"))


def test_disable_fusions_env_switch():
    code = ("import determined_amd.ops as o; "
            "print(o.fusion_enabled('split_grad'), o.fusion_enabled('stem_conv'), o.fusion_enabled('avgpool'), "
            "o.fusion_enabled('igemm_conv'), o.fusion_enabled('conv_stats'), o.fusion_enabled('bn_conv'), "
            "o.fusion_enabled('bn_prologue'), o.fusion_enabled('bn_lazy_bwd'))")
    env = dict(os.environ, PYTHONPATH=ROOT, DAMD_DISABLE_FUSIONS="split_grad, stem_conv,igemm_conv,bn_prologue")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True)
    assert out.stdout.split() == ["False", "False", "True", "False", "True", "True", "False", "True"]


def test_igemm_conv_path_falls_back_on_cpu():
    from determined_amd.ops.conv import conv2d, conv_bn_input, igemm_fusable

    torch.manual_seed(0)
    conv = torch.nn.Conv2d(64, 64, 3, padding=1, bias=False)
    x = torch.randn(2, 64, 7, 7, requires_grad=True)
    assert not igemm_fusable(conv, x)
    y, part = conv_bn_input(conv, x)
    assert part is None
    torch.testing.assert_close(y, conv(x))
    torch.testing.assert_close(conv2d(conv, x), conv(x))


def test_igemm_conv_skips_modules_with_hooks():
    from determined_amd.ops.conv import _plain_module

    conv = torch.nn.Conv2d(64, 64, 1, bias=False)
    assert _plain_module(conv)
    h = conv.register_forward_hook(lambda m, i, o: None)
    assert not _plain_module(conv)
    h.remove()
    conv.register_forward_pre_hook(lambda m, i: None)
    assert not _plain_module(conv)
    wn = torch.nn.utils.parametrizations.weight_norm(torch.nn.Conv2d(64, 64, 1, bias=False))
    assert not _plain_module(wn)


def test_resnet_forward_with_stats_path_matches_plain_on_cpu():
    """The block forwards thread (y, stats_part) through conv_bn_input; on CPU the parts are None
    and the result equals the module composition."""
    from determined_amd.models.resnet import resnet18

    torch.manual_seed(0)
    m = resnet18(num_classes=10).train()
    x = torch.randn(2, 3, 32, 32)
    out = m(x)
    assert out.shape == (2, 10) and torch.isfinite(out).all()


def test_chained_resnet_forward_equals_per_block_on_cpu(monkeypatch):
    """The fused block chain (models/resnet.py _chain_blocks) is the exact per-block composition
    on CPU (its fused autograd nodes only engage on the GPU)."""
    import determined_amd.ops as ops
    from determined_amd.models.resnet import resnet50

    torch.manual_seed(0)
    m = resnet50(num_classes=10).train()
    x = torch.randn(2, 3, 64, 64)
    outs = []
    for disabled in (frozenset(), frozenset({"bn_conv"})):
        monkeypatch.setattr(ops, "_DISABLED", disabled)
        m.zero_grad()
        out = m(x)
        out.square().sum().backward()
        outs.append((out.detach(), m.layer2[1].conv2.weight.grad.clone()))
    torch.testing.assert_close(outs[0][0], outs[1][0])
    torch.testing.assert_close(outs[0][1], outs[1][1])


def test_conv_exclude_spec_parsing():
    from determined_amd.ops.conv import _parse_exclude

    ex = _parse_exclude("wgrad:8-10, *:14,fwd:miopen,bogus")
    assert ex == frozenset({("wgrad", 8), ("wgrad", 9), ("wgrad", 10), ("*", 14), ("fwd", "miopen")})


def test_conv_tune_db_roundtrip(tmp_path, monkeypatch):
    import determined_amd.ops.conv as conv

    monkeypatch.setattr(conv, "_TUNE", {("fwd", (512, 64, 56, 56), (64, 64, 3, 3), 1, 1): 7,
                                        ("wgrad", (8, 64, 9, 9), (64, 64, 3, 3), 1, 1): "h1",
                                        ("fwd_pro_pays", (512, 64, 56, 56), (64, 64, 3, 3)): True})
    p = tmp_path / "db.jsonl"
    assert conv.save_tune_db(str(p)) == 3
    saved = dict(conv._TUNE)
    monkeypatch.setattr(conv, "_TUNE", {})
    assert conv.load_tune_db(str(p)) == 3
    assert conv._TUNE == saved
    # a shipped choice is used only if it is one of the candidates of this build
    monkeypatch.setattr(conv, "_DB_LOADED", True)
    assert conv._pick(("fwd", (512, 64, 56, 56), (64, 64, 3, 3), 1, 1), {3: None, 7: None}, 3) == 7


def test_flip_weight_matches_flip_transpose():
    """The dgrad weights (flipped taps, transposed channels, channels-last) from the single gather
    equal flip(2, 3).transpose(0, 1)."""
    from determined_amd.ops.conv import _flip_weight

    for shp in [(64, 32, 3, 3), (128, 64, 1, 1), (8, 16, 7, 7)]:
        w = torch.randn(*shp).contiguous(memory_format=torch.channels_last)
        ref = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)
        out = _flip_weight(w)
        assert torch.equal(out, ref) and out.is_contiguous(memory_format=torch.channels_last)


def test_lazy_bn_residual_and_strided_grad_fallbacks_on_cpu():
    """Off the GPU kernels a LazyBNResidual is materialised (bn(y)) before the plain composition,
    and a compact stride-2 gradient expands to the full grid with zeros at the odd pixels."""
    from determined_amd.ops.bn import BatchNormAct2d
    from determined_amd.ops.conv import LazyBNResidual, _StridedGrad, bn_act_conv

    torch.manual_seed(0)
    bn, bnr = BatchNormAct2d(8), BatchNormAct2d(8, act=False)
    conv = torch.nn.Conv2d(8, 4, 1, bias=False)
    y, yr = torch.randn(2, 8, 5, 5), torch.randn(2, 8, 5, 5)
    a, z, part = bn_act_conv(bn, y, None, LazyBNResidual(yr, None, bnr), conv)
    bn2, bnr2 = BatchNormAct2d(8), BatchNormAct2d(8, act=False)
    a_ref = bn2(y, bnr2(yr))
    torch.testing.assert_close(a, a_ref)
    torch.testing.assert_close(z, conv(a_ref))
    c = torch.randn(2, 3, 3, 3)
    full = _StridedGrad.materialise(c, (2, 3, 5, 5))
    assert torch.equal(full[:, :, ::2, ::2], c) and full[:, :, 1::2].abs().sum() == 0 and full[:, :, :, 1::2].abs().sum() == 0
