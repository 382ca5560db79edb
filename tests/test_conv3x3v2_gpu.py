"""Zero-padded-halo 3x3 kernels (csrc/conv3x3v2.hip, the conv configs after the conv_igemm.hip ones)
vs fp32 PyTorch references: plain forward (+ BN statistics), BN+ReLU prologue forward (`a` written),
input gradient with the BN-backward epilogue (bit mask / recomputed ReLU), and with the deferred
BN-backward apply prologue; multi channel-block / multi co-tile / non-square geometries; run-to-run
identity (a missing barrier on the halo double buffer would show as run-to-run differences)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last


@pytest.fixture(scope="module")
def ext():
    import determined_amd.ops as ops

    return ops.ext()


def _v2_cfgs(ext, x, w):
    from determined_amd.ops import conv as C  # noqa: F401  (same cfg numbering as the tuner's)

    base = ext.conv_num_cfgs() - ext.conv_v2_num_cfgs()
    return [c for c in range(base, ext.conv_num_cfgs()) if ext.conv_supported(x, w, c, 1, 1)]


def _rand(*shape, scale=1.0):
    return (torch.randn(*shape, device="cuda") * scale).to(torch.bfloat16).contiguous(memory_format=CL)


# (n, cin, cout, H, W): one v2 config each plus multi channel-block (64-channel blocks 2, 4, 8: the weight ring
# wraps at different taps per unit) / co-tile and non-square cases
SHAPES = [(2, 64, 64, 56, 56), (1, 128, 128, 8, 56), (3, 128, 128, 28, 28), (2, 64, 256, 12, 28),
          (3, 128, 128, 14, 14), (2, 256, 256, 14, 14), (1, 256, 64, 4, 56), (2, 128, 512, 8, 28),
          (1, 256, 64, 8, 56), (2, 256, 128, 14, 28)]


@pytest.mark.parametrize("shape", SHAPES)
def test_v2_forward_and_stats(ext, shape):
    n, cin, cout, H, W = shape
    torch.manual_seed(0)
    x = _rand(n, cin, H, W)
    w = _rand(cout, cin, 3, 3, scale=(cin * 9) ** -0.5)
    ref = F.conv2d(x.float(), w.float(), padding=1)
    cfgs = _v2_cfgs(ext, x, w)
    assert cfgs, "shape not served by a v2 config"
    for cfg in cfgs:
        y, part = ext.conv_fwd(x, w, 1, 1, True, cfg, 0)
        torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
        tol = 2e-3 * ref.abs().sum((0, 2, 3)).max().item()
        torch.testing.assert_close(part[:, 0].sum(0), ref.sum((0, 2, 3)), rtol=1e-3, atol=tol)
        torch.testing.assert_close(part[:, 1].sum(0), (ref * ref).sum((0, 2, 3)), rtol=2e-3,
                                   atol=2e-3 * (ref * ref).sum((0, 2, 3)).max().item())
        y0, _ = ext.conv_fwd(x, w, 1, 1, False, cfg, 0)  # no-epilogue variant
        assert torch.equal(y0, y)
        for _ in range(3):
            assert torch.equal(ext.conv_fwd(x, w, 1, 1, True, cfg, 0)[0], y)


@pytest.mark.parametrize("shape", SHAPES)
def test_v2_bn_relu_prologue(ext, shape):
    n, cin, cout, H, W = shape
    torch.manual_seed(1)
    y = _rand(n, cin, H, W)
    w = _rand(cout, cin, 3, 3, scale=(cin * 9) ** -0.5)
    a_ref, stats, _ = ext.bn_act_fwd(y, torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2,
                                     None, None, 0.0, 1e-5, None, True, False, None)
    z_ref = F.conv2d(a_ref.float(), w.float(), padding=1)
    cfgs = [c for c in _v2_cfgs(ext, y, w) if ext.conv_pro_supported(y, w, c)]
    assert cfgs
    for cfg in cfgs:
        z, part, a, mask = ext.conv_bnact_fwd(y, w, None, stats, False, cfg, None)
        torch.testing.assert_close(a, a_ref, rtol=0, atol=0)  # every pixel of `a` written, exactly
        torch.testing.assert_close(z.float(), z_ref, rtol=2e-2, atol=2e-2 * z_ref.abs().max().item())
        tol = 2e-3 * z_ref.abs().sum((0, 2, 3)).max().item()
        torch.testing.assert_close(part[:, 0].sum(0), z_ref.sum((0, 2, 3)), rtol=1e-3, atol=tol)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("masked", [False, True])
def test_v2_dgrad_bn_epilogue(ext, shape, masked):
    """dz = dX * relu-mask (bit mask of a residual BN, or recomputed from yb) + BN-backward partials."""
    n, cin, cout, H, W = shape
    torch.manual_seed(2)
    w = _rand(cout, cin, 3, 3, scale=(cin * 9) ** -0.5)
    wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=CL)  # [cin, cout, 3, 3]
    g = _rand(n, cout, H, W)
    yb = _rand(n, cin, H, W)
    res = _rand(n, cin, H, W) if masked else None
    a, stats, mask = ext.bn_act_fwd(yb, torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2,
                                    None, None, 0.0, 1e-5, res, True, True, None)
    da = torch.nn.grad.conv2d_input(yb.shape, w.float(), g.float(), padding=1)
    ref = da * (a.float() > 0)
    cen = yb.float() - stats[0].view(1, -1, 1, 1)
    cfgs = _v2_cfgs(ext, g, wt)
    if not cfgs:  # e.g. 64 input-gradient channels at W = 28 (that config's co tile is 128)
        pytest.skip("no v2 config serves this input gradient")
    for cfg in cfgs:
        dz, part = ext.conv_dgrad_bn(g, wt, 1, cfg, None, yb, mask if masked else None, stats, None, None)
        torch.testing.assert_close(dz.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
        dzf = dz.float()
        torch.testing.assert_close(part[:, 0].sum(0), dzf.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
        torch.testing.assert_close(part[:, 1].sum(0), (dzf * cen).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("shape", SHAPES)
def test_v2_dgrad_deferred_bn_apply(ext, shape):
    """PRO 2: the operand dy = A*dz + B*y + Cc formed in the halo staging (and returned) == the kernel run
    on the explicitly applied dy; run-to-run identical."""
    n, cin, cout, H, W = shape
    torch.manual_seed(3)
    w = _rand(cout, cin, 3, 3, scale=(cin * 9) ** -0.5)
    wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=CL)
    dzn = _rand(n, cout, H, W)
    yn = torch.randn_like(dzn)
    coef = torch.randn(3, cout, device="cuda").contiguous()
    yb = _rand(n, cin, H, W)
    _, stb, _ = ext.bn_act_fwd(yb, torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2,
                               None, None, 0.0, 1e-5, None, True, False, None)
    dy_ref = ext.bn_bwd_apply_coef(dzn, yn, coef)
    cfgs = [c for c in _v2_cfgs(ext, dzn, wt) if ext.conv_pro_supported(dzn, wt, c)]
    if not cfgs:
        pytest.skip("no v2 config serves this input gradient")
    for cfg in cfgs:
        dz_ref, part_ref = ext.conv_dgrad_bn(dy_ref, wt, 1, cfg, None, yb, None, stb, None, None)
        dz, part, dy = ext.conv_dgrad_bn(dzn, wt, 1, cfg, None, yb, None, stb, yn, coef)
        torch.testing.assert_close(dy.float(), dy_ref.float(), rtol=1e-2, atol=1e-2)
        torch.testing.assert_close(dz.float(), dz_ref.float(), rtol=1e-2, atol=1e-2)
        torch.testing.assert_close(part, part_ref, rtol=1e-3, atol=1e-2)
        for _ in range(4):
            dz2, _, dy2 = ext.conv_dgrad_bn(dzn, wt, 1, cfg, None, yb, None, stb, yn, coef)
            assert torch.equal(dz2, dz) and torch.equal(dy2, dy)


def test_v2_refuses_unsupported_geometry(ext):
    """W not one of the compiled widths, H not a multiple of the tile rows, stride 2: no v2 config."""
    w = _rand(64, 64, 3, 3)
    base = ext.conv_num_cfgs() - ext.conv_v2_num_cfgs()
    for shape in [(1, 64, 56, 30), (1, 64, 10, 56), (1, 64, 28, 27)]:
        x = _rand(*shape)
        assert not any(ext.conv_supported(x, w, c, 1, 1) for c in range(base, ext.conv_num_cfgs()))
    x = _rand(1, 64, 56, 56)
    assert not any(ext.conv_supported(x, w, c, 2, 1) for c in range(base, ext.conv_num_cfgs()))


@pytest.mark.parametrize("shape", [(2, 64, 64, 56, 56), (1, 128, 64, 8, 56), (2, 128, 128, 28, 28),
                                   (1, 64, 192, 14, 28), (2, 256, 128, 14, 14), (3, 64, 64, 14, 14),
                                   (3, 128, 64, 7, 7)])
def test_v2_wgrad_matches_fp32(ext, shape):
    """conv3x3v2.hip's whole-row-tile weight gradient (wgrad3x3 cfgs >= 2: transposed LDS reads of
    8-channel planes, zero border from out-of-range DMA offsets) vs fp32, bf16 and fp32 weight outputs,
    run-to-run identical (deterministic split reduction)."""
    n, cin, cout, h, wd = shape
    torch.manual_seed(11)
    x = _rand(n, cin, h, wd)
    dy = _rand(n, cout, h, wd)
    w = _rand(cout, cin, 3, 3)
    ref = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), stride=1, padding=1)
    cfgs = [c for c in range(2, ext.wgrad3x3_num_cfgs()) if ext.wgrad3x3_supported(x, dy, w, c)]
    assert cfgs, "shape not served by a v2 weight-gradient config"
    for cfg in cfgs:
        dw = ext.conv3x3_wgrad(x, dy, w, cfg, 0)
        assert dw.shape == w.shape and dw.dtype == w.dtype and dw.is_contiguous(memory_format=CL)
        torch.testing.assert_close(dw.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
        dw32 = ext.conv3x3_wgrad(x, dy, w.float(), cfg, 0)
        torch.testing.assert_close(dw32, ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
        assert torch.equal(ext.conv3x3_wgrad(x, dy, w.float(), cfg, 0), dw32)
