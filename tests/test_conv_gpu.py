"""Implicit-GEMM convolution kernels (csrc/conv_igemm.hip) vs fp32 PyTorch references."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ext():
    import determined_amd.ops as ops

    return ops.ext()


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


SHAPES = [  # (n, cin, cout, k, stride, hw)
    (2, 64, 64, 1, 1, 9),
    (3, 64, 128, 3, 1, 7),
    (2, 128, 64, 3, 2, 11),
    (1, 256, 256, 1, 2, 14),
    (2, 192, 128, 3, 1, 5),
    (2, 64, 64, 3, 1, 30),
    (1, 128, 256, 3, 1, 57),
]


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_fwd_and_stats_match_fp32(ext, shape):
    n, cin, cout, k, st, hw = shape
    pad = k // 2
    torch.manual_seed(0)
    x = cl(torch.randn(n, cin, hw, hw, device="cuda").to(torch.bfloat16))
    w = cl((torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5).to(torch.bfloat16))
    ref = F.conv2d(x.float(), w.float(), stride=st, padding=pad)
    for cfg in range(ext.conv_num_cfgs()):
        if not ext.conv_supported(x, w, cfg, st, pad):
            continue
        y, part = ext.conv_fwd(x, w, st, pad, True, cfg, 0)
        assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
        torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
        # statistics of the fp32 conv outputs (before the bf16 store)
        tol = 2e-3 * ref.abs().sum((0, 2, 3)).max().item()
        torch.testing.assert_close(part[:, 0].sum(0), ref.sum((0, 2, 3)), rtol=1e-3, atol=tol)
        torch.testing.assert_close(part[:, 1].sum(0), (ref * ref).sum((0, 2, 3)), rtol=2e-3,
                                   atol=2e-3 * (ref * ref).sum((0, 2, 3)).max().item())
        # a forced small group count exercises several pixel tiles per block (persistent loop)
        y2, _ = ext.conv_fwd(x, w, st, pad, False, cfg, 1)
        torch.testing.assert_close(y2, y, rtol=0, atol=0)


@pytest.mark.parametrize("shape", [s for s in SHAPES if s[4] == 1])
def test_conv_dgrad_via_flipped_weights(ext, shape):
    """stride-1 input gradient = forward conv of dY with flipped, transposed weights."""
    n, cin, cout, k, st, hw = shape
    pad = k // 2
    torch.manual_seed(1)
    x = torch.randn(n, cin, hw, hw, device="cuda")
    w = (torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5).to(torch.bfloat16)
    dy = cl(torch.randn(n, cout, hw, hw, device="cuda").to(torch.bfloat16))
    ref = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), stride=1, padding=pad)
    wt = cl(w.flip(2, 3).transpose(0, 1))
    if not ext.conv_supported(dy, wt, -1, 1, k - 1 - pad):
        pytest.skip("channel count not covered by a config")
    dx, _ = ext.conv_fwd(dy, wt, 1, k - 1 - pad, False, -1, 0)
    torch.testing.assert_close(dx.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())


@pytest.mark.parametrize("shape", SHAPES + [(2, 64, 128, 3, 1, 23), (1, 128, 64, 1, 1, 40), (2, 256, 512, 3, 1, 9),
                                   (3, 512, 256, 1, 1, 12)])
def test_conv_wgrad_matches_fp32(ext, shape):
    n, cin, cout, k, st, hw = shape
    pad = k // 2
    torch.manual_seed(2)
    x = cl(torch.randn(n, cin, hw, hw, device="cuda").to(torch.bfloat16))
    w = cl(torch.randn(cout, cin, k, k, device="cuda").to(torch.bfloat16))
    oh = (hw + 2 * pad - k) // st + 1
    dy = cl(torch.randn(n, cout, oh, oh, device="cuda").to(torch.bfloat16))
    ref = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), stride=st, padding=pad)
    ran = 0
    for cfg in range(ext.wgrad_num_cfgs()):
        if not ext.wgrad_supported(x, dy, cout, cfg):
            continue
        for splits in (0, 1, 3):
            dw = ext.conv_wgrad(x, dy, w, st, pad, cfg, splits)
            assert dw.shape == w.shape and dw.dtype == w.dtype
            torch.testing.assert_close(dw.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
        ran += 1
    assert ran > 0
    cfg0 = 0 if ext.wgrad_supported(x, dy, cout, 0) else 3
    dw32 = ext.conv_wgrad(x, dy, w.float(), st, pad, cfg0, 0)
    assert dw32.dtype == torch.float32
    torch.testing.assert_close(dw32, ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())


SK_TWIN = {14: 1, 15: 5, 16: 3, 17: 4, 18: 6, 19: 7, 20: 8, 21: 9}  # stream-K config -> whole-tile twin


@pytest.mark.parametrize("shape", [(16, 256, 256, 3, 1, 14), (32, 512, 512, 3, 1, 7), (8, 1024, 256, 1, 1, 14),
                                   (2, 64, 64, 3, 1, 9), (24, 2048, 512, 1, 1, 7), (4, 128, 128, 3, 1, 28)])
def test_stream_k_configs_match_whole_tile_twins(ext, shape):
    """Stream-K work split (tiles computed in segments by consecutive blocks, fp32 slabs handed
    over in-launch): output and BN statistics vs fp32 and vs the same tile run whole; bitwise
    reproducible launch to launch; no hand-off ever times out."""
    n, cin, cout, k, st, hw = shape
    pad = k // 2
    torch.manual_seed(5)
    x = cl(torch.randn(n, cin, hw, hw, device="cuda").to(torch.bfloat16))
    w = cl((torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5).to(torch.bfloat16))
    ref = F.conv2d(x.float(), w.float(), stride=st, padding=pad)
    ran = 0
    for cfg, twin in SK_TWIN.items():
        assert ext.conv_sk_cfg(cfg) and not ext.conv_sk_cfg(twin)
        if not ext.conv_supported(x, w, cfg, st, pad):
            continue
        y, part = ext.conv_fwd(x, w, st, pad, True, cfg, 0)
        torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
        yt, _ = ext.conv_fwd(x, w, st, pad, False, twin, 0)
        torch.testing.assert_close(y.float(), yt.float(), rtol=1e-2, atol=1e-2 * ref.abs().max().item())
        tol = 2e-3 * ref.abs().sum((0, 2, 3)).max().item()
        torch.testing.assert_close(part[:, 0].sum(0), ref.sum((0, 2, 3)), rtol=1e-3, atol=tol)
        y2, part2 = ext.conv_fwd(x, w, st, pad, True, cfg, 0)
        assert torch.equal(y2, y) and torch.equal(part2, part)
        ran += 1
    assert ran > 0
    torch.cuda.synchronize()
    assert ext.conv_sk_timeouts(x) == 0


@pytest.mark.parametrize("shape", [(2, 64, 64, 9), (3, 128, 128, 7), (1, 256, 128, 14), (2, 64, 128, 23),
                                   (4, 512, 512, 7), (1, 128, 64, 57)])
def test_conv3x3_halo_wgrad_matches_fp32(ext, shape):
    """3x3 halo weight gradient (zero-padded pixel grid, 9 taps from one staged halo) vs fp32,
    every config and forced split counts; bf16 and fp32 weight outputs."""
    n, cin, cout, hw = shape
    torch.manual_seed(7)
    x = cl(torch.randn(n, cin, hw, hw, device="cuda").to(torch.bfloat16))
    w = cl(torch.randn(cout, cin, 3, 3, device="cuda").to(torch.bfloat16))
    dy = cl(torch.randn(n, cout, hw, hw, device="cuda").to(torch.bfloat16))
    ref = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), stride=1, padding=1)
    ran = 0
    for cfg in (0, 1):
        if not ext.wgrad3x3_supported(x, dy, w, cfg):
            continue
        for splits in (0, 1, 5):
            dw = ext.conv3x3_wgrad(x, dy, w, cfg, splits)
            assert dw.shape == w.shape and dw.dtype == w.dtype and dw.is_contiguous(memory_format=torch.channels_last)
            torch.testing.assert_close(dw.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
        dw32 = ext.conv3x3_wgrad(x, dy, w.float(), cfg, 0)
        torch.testing.assert_close(dw32, ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
        ran += 1
    assert ran > 0


@pytest.mark.parametrize("shape", [(8, 128, 128, 56), (4, 256, 256, 28), (4, 512, 512, 14), (2, 64, 128, 16)])
def test_stride2_3x3_dgrad_by_phases(ext, shape):
    """The four-phase stride-2 3x3 input gradient (ops/conv.py _dgrad_s2_phases) against an fp32
    reference, for every tile config that supports the phase geometry."""
    from determined_amd.ops import conv as C

    n, cin, cout, hw = shape
    g = torch.Generator(device="cuda")
    g.manual_seed(hw)
    w = (torch.randn(cout, cin, 3, 3, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    dy = torch.randn(n, cout, hw // 2, hw // 2, device="cuda", generator=g).to(torch.bfloat16)
    dy = dy.contiguous(memory_format=torch.channels_last)
    ref = torch.nn.grad.conv2d_input((n, cin, hw, hw), w.float(), dy.float(), stride=2, padding=1)
    cfgs = C._phase_cfgs(ext, dy, w)
    assert cfgs
    for c in cfgs:
        dx = C._dgrad_s2_phases(ext, dy, w, (n, cin, hw, hw), c)
        err = ((dx.float() - ref).norm() / ref.norm()).item()
        assert err < 1e-2, (c, err)


@pytest.mark.parametrize("k,st", [(3, 2), (1, 2)])
def test_conv_fwd_input_over_2gib(ext, k, st):
    """inputs above 2^31 bytes (the batch-2048 default has several) -- the kernel's im2col
    byte offsets are unsigned 32-bit; images past the 2 GiB mark (and the padded borders, whose tap
    offsets lie before the tensor) are compared with a chunked fp32 reference."""
    n, cin, cout, hw = 1400, 256, 64, 56  # 2.25 GB of bf16 input
    pad = k // 2
    torch.manual_seed(0)
    x = torch.empty(n, hw, hw, cin, device="cuda", dtype=torch.bfloat16).normal_().permute(0, 3, 1, 2)
    assert x.is_contiguous(memory_format=torch.channels_last) and x.numel() * 2 > 2 ** 31
    w = cl((torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5).to(torch.bfloat16))
    cfgs = [c for c in range(ext.conv_num_cfgs()) if ext.conv_supported(x, w, c, st, pad)]
    assert cfgs
    for cfg in cfgs[:3]:
        y, _ = ext.conv_fwd(x, w, st, pad, False, cfg, 0)
        for lo in (0, 1330, n - 8):  # before, across and after the 2^31-byte mark
            ref = F.conv2d(x[lo:lo + 8].float(), w.float(), stride=st, padding=pad)
            torch.testing.assert_close(y[lo:lo + 8].float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
        del y
    torch.cuda.empty_cache()


def test_1x1_wgrad_gemm_candidate_matches_fp32(ext, monkeypatch):
    """The hipBLASLt candidate of the 1x1 stride-1 weight gradient (dW = dY^T X over the pixels)
    against fp32, in the layout and dtype of the other candidates."""
    from determined_amd.ops import conv as C

    torch.manual_seed(3)
    x = cl(torch.randn(4, 128, 14, 14, device="cuda").to(torch.bfloat16))
    dy = cl(torch.randn(4, 256, 14, 14, device="cuda").to(torch.bfloat16))
    w = cl(torch.randn(256, 128, 1, 1, device="cuda").to(torch.bfloat16))
    ref = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), stride=1, padding=0)
    picked = []
    monkeypatch.setattr(C, "_pick", lambda key, cands, default=None: picked.append(sorted(map(str, cands))) or "gemm")
    dw = C._wgrad(dy, x, w, 1, 0)
    assert "gemm" in picked[0]
    assert dw.shape == w.shape and dw.dtype == w.dtype and dw.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(dw.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
    # stride 2 (the downsample shortcut): the even pixels of x
    dy2 = cl(torch.randn(4, 256, 7, 7, device="cuda").to(torch.bfloat16))
    ref2 = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy2.float(), stride=2, padding=0)
    dw2 = C._wgrad(dy2, x, w, 2, 0)
    torch.testing.assert_close(dw2.float(), ref2, rtol=2e-2, atol=2e-2 * ref2.abs().max().item())
