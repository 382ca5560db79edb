"""Numerics of the hand-written HIP kernels vs plain PyTorch fp32 references (run on MI355X)."""

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ops():
    import determined_amd.ops as ops

    ops.ext()  # must load: these tests exist to exercise the native path
    return ops


def _params(shapes, dtype=torch.float32, seed=0):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    ps = [torch.nn.Parameter(torch.randn(s, device="cuda", generator=g).to(dtype)) for s in shapes]
    for p in ps:
        p.grad = torch.randn(p.shape, device="cuda", generator=g).to(dtype)
    return ps


SHAPES = [(3,), (17, 5), (1024,), (64, 3, 7, 7), (257, 129), (40000,)]


@pytest.mark.parametrize("adam_w_mode", [True, False])
def test_fused_adamw_matches_torch(ops, adam_w_mode):
    ref = _params(SHAPES)
    ours = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    for a, b in zip(ours, ref):
        a.grad = b.grad.clone()
    Ref = torch.optim.AdamW if adam_w_mode else torch.optim.Adam
    o_ref = Ref(ref, lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=0.1)
    o_ours = ops.FusedAdamW(ours, lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=0.1, adam_w_mode=adam_w_mode)
    for step in range(5):
        for a, b in zip(ours, ref):
            g = torch.randn_like(b) * (step + 1)
            a.grad.copy_(g)
            b.grad.copy_(g)
        o_ref.step()
        o_ours.step()
    for a, b in zip(ours, ref):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_fused_adamw_master_weights_bf16(ops):
    ref = _params(SHAPES)
    ours = [torch.nn.Parameter(p.detach().to(torch.bfloat16)) for p in ref]
    for p in ref:
        p.data = p.data.to(torch.bfloat16).float()
    o_ref = torch.optim.AdamW(ref, lr=1e-3, weight_decay=0.01)
    o_ours = ops.FusedAdamW(ours, lr=1e-3, weight_decay=0.01, master_weights=True)
    for _ in range(4):
        for a, b in zip(ours, ref):
            g = torch.randn_like(b).to(torch.bfloat16)
            a.grad = g.clone()
            b.grad = g.float()
        o_ref.step()
        o_ours.step()
    for a, b in zip(ours, ref):
        st = o_ours.state[a]
        torch.testing.assert_close(st["master"], b.detach(), rtol=1e-5, atol=1e-6)
        # the bf16 param is exactly the RNE rounding of its own fp32 master (which matches the
        # reference to 1e-5; comparing against the reference's rounding flips 1 ulp at ties)
        torch.testing.assert_close(a.detach().float(), st["master"].to(torch.bfloat16).float(), rtol=0, atol=0)


@pytest.mark.parametrize("nesterov,dampening", [(False, 0.0), (True, 0.0), (False, 0.1)])
def test_fused_sgd_matches_torch(ops, nesterov, dampening):
    ref = _params(SHAPES, seed=3)
    ours = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    o_ref = torch.optim.SGD(ref, lr=0.05, momentum=0.9, dampening=dampening, weight_decay=1e-3, nesterov=nesterov)
    o_ours = ops.FusedSGD(ours, lr=0.05, momentum=0.9, dampening=dampening, weight_decay=1e-3, nesterov=nesterov)
    for _ in range(4):
        for a, b in zip(ours, ref):
            g = torch.randn_like(b)
            a.grad = g.clone()
            b.grad = g.clone()
        o_ref.step()
        o_ours.step()
    for a, b in zip(ours, ref):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_fused_sgd_channels_last_grads(ops):
    w = torch.nn.Parameter(torch.randn(64, 32, 3, 3, device="cuda").to(memory_format=torch.channels_last))
    w.grad = torch.randn_like(w)
    ref = torch.nn.Parameter(w.detach().clone())
    ref.grad = w.grad.clone()
    o = ops.FusedSGD([w], lr=0.1, momentum=0.9)
    r = torch.optim.SGD([ref], lr=0.1, momentum=0.9)
    o.step()
    r.step()
    torch.testing.assert_close(w, ref)


def test_fused_clip_and_integrated_clip(ops):
    ref = _params(SHAPES, seed=5)
    ours = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    for a, b in zip(ours, ref):
        a.grad = b.grad.clone()
    n_ref = torch.nn.utils.clip_grad_norm_(ref, 1.0)
    n_ours = ops.fused_clip_grad_norm_(ours, 1.0)
    torch.testing.assert_close(n_ours.reshape(()), n_ref, rtol=1e-5, atol=1e-5)
    for a, b in zip(ours, ref):
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-5, atol=1e-6)
    # integrated: clip inside FusedSGD.step must equal clip-then-step
    ref2 = _params(SHAPES, seed=6)
    ours2 = [torch.nn.Parameter(p.detach().clone()) for p in ref2]
    for a, b in zip(ours2, ref2):
        a.grad = b.grad.clone()
    torch.nn.utils.clip_grad_norm_(ref2, 0.5)
    torch.optim.SGD(ref2, lr=0.1).step()
    o = ops.FusedSGD(ours2, lr=0.1)
    o.set_grad_clipping(0.5)
    o.step()
    for a, b in zip(ours2, ref2):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_scaler_skips_on_inf_without_sync(ops):
    ps = _params([(1000,), (33,)])
    before = [p.detach().clone() for p in ps]
    opt = ops.FusedAdamW(ps, lr=1e-2)
    scaler = ops.DeviceGradScaler(init_scale=1024.0, growth_interval=1)
    loss = torch.zeros((), device="cuda", requires_grad=True)
    scaler.scale(loss)
    ps[0].grad[3] = float("inf")
    scaler.step(opt)
    scaler.update()
    for p, b in zip(ps, before):
        torch.testing.assert_close(p.detach(), b)
    assert scaler.get_scale() == 512.0
    assert float(opt._step_tensor(ps[0].device).item()) == 0.0
    ps[0].grad.zero_()
    scaler.step(opt)
    scaler.update()
    assert float(opt._step_tensor(ps[0].device).item()) == 1.0
    assert scaler.get_scale() == 1024.0


def test_scaler_unscale_then_clip_then_step(ops):
    """use_amp's order: unscale_ before clipping, then step applies only the skip decision."""
    ref = _params([(1000,), (33,)], seed=9)
    ps = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    for a, b in zip(ps, ref):
        a.grad = b.grad * 256.0  # gradients of a loss scaled by 256
    torch.nn.utils.clip_grad_norm_(ref, 0.5)
    torch.optim.SGD(ref, lr=0.1).step()
    opt = ops.FusedSGD(ps, lr=0.1)
    scaler = ops.DeviceGradScaler(init_scale=256.0)
    scaler.scale(torch.zeros((), device="cuda"))
    scaler.unscale_(opt)
    with pytest.raises(RuntimeError):
        scaler.unscale_(opt)
    torch.nn.utils.clip_grad_norm_(ps, 0.5)
    scaler.step(opt)
    scaler.update()
    for a, b in zip(ps, ref):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    # a non-finite gradient seen by unscale_ skips the step
    before = [p.detach().clone() for p in ps]
    ps[1].grad.fill_(float("nan"))
    scaler.unscale_(opt)
    scaler.step(opt)
    scaler.update()
    for p, b in zip(ps, before):
        torch.testing.assert_close(p.detach(), b)
    assert scaler.get_scale() == 128.0


def _ref_ln(x, w, b, eps, rms):
    xf = x.float()
    if rms:
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    else:
        y = torch.nn.functional.layer_norm(xf, (x.shape[-1],), w.float(), b.float() if b is not None else None, eps)
    return y


@pytest.mark.parametrize("H", [64, 768, 1000, 1024, 1600, 4096, 8192])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rms", [False, True])
def test_norm_fwd_bwd(ops, H, dtype, rms):
    torch.manual_seed(H)
    rows = 257
    x = (torch.randn(rows, H, device="cuda") * 3 + 1).to(dtype).requires_grad_(True)
    w = (torch.rand(H, device="cuda") + 0.5).to(dtype).requires_grad_(True)
    b = None if rms else (torch.randn(H, device="cuda") * 0.1).to(dtype).requires_grad_(True)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    br = None if b is None else b.detach().float().requires_grad_(True)
    y = ops.rms_norm(x, w, 1e-5) if rms else ops.layer_norm(x, w, b, 1e-5)
    yr = _ref_ln(xr, wr, br, 1e-5, rms)
    tol = dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(y.float(), yr, **tol)
    gy = torch.randn_like(yr)
    (y.float() * gy).sum().backward()
    (yr * gy).sum().backward()
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)
    gtol = dict(rtol=3e-2, atol=5e-1) if dtype == torch.bfloat16 else dict(rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(w.grad.float(), wr.grad, **gtol)
    if b is not None:
        torch.testing.assert_close(b.grad.float(), br.grad, **gtol)


def test_ddp_single_rank_grads_match(ops):
    from determined_amd.models.resnet import resnet18
    from determined_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    m = resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last)
    m_ref = copy.deepcopy(m)
    ddp = DistributedDataParallel(m, bucket_cap_mb=1)
    x = torch.randn(4, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    for it in range(2):
        ddp.zero_grad()
        m_ref.zero_grad()
        ddp(x).sum().backward()
        ddp.finish()
        m_ref(x).sum().backward()
        for (n, p), (_, q) in zip(m.named_parameters(), m_ref.named_parameters()):
            torch.testing.assert_close(p.grad, q.grad, rtol=1e-4, atol=1e-4, msg=n)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("H", [64, 1024, 1600])
def test_residual_dropout_layernorm_fused(dtype, H):
    """s = x + dropout(b); y = LN(s): fused kernel vs fp32 PyTorch (p=0 exact path; p>0 checks
    the keep-mask statistics and that fwd/bwd use the same mask)."""
    from determined_amd.ops.norm import FusedLayerNorm

    torch.manual_seed(0)
    ln = FusedLayerNorm(H).cuda().to(dtype)
    with torch.no_grad():
        ln.weight.uniform_(0.5, 1.5)
        ln.bias.uniform_(-0.2, 0.2)
    x = torch.randn(3, 37, H, device="cuda", dtype=dtype, requires_grad=True)
    b = torch.randn(3, 37, H, device="cuda", dtype=dtype, requires_grad=True)
    s, y = ln(x, branch=b, p=0.0)
    xr, br = x.detach().float().requires_grad_(True), b.detach().float().requires_grad_(True)
    sr = xr + br
    yr = torch.nn.functional.layer_norm(sr, (H,), ln.weight.float(), ln.bias.float(), ln.eps)
    tol = dict(rtol=2e-2, atol=3e-2) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(s.float(), sr, **tol)
    torch.testing.assert_close(y.float(), yr, **tol)
    gs, gy = torch.randn_like(sr), torch.randn_like(yr)
    torch.autograd.backward([s, y], [gs.to(dtype), gy.to(dtype)])
    torch.autograd.backward([sr, yr], [gs, gy])
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)
    torch.testing.assert_close(b.grad.float(), br.grad, **tol)
    # dropout: about p of the branch is dropped, kept elements scaled by 1/(1-p), and the
    # branch gradient flows exactly through the kept elements
    p = 0.25
    x2 = torch.zeros(64, H, device="cuda", dtype=dtype)
    b2 = torch.ones(64, H, device="cuda", dtype=dtype, requires_grad=True)
    ln.train()
    s2, y2 = ln(x2, branch=b2, p=p)
    kept = s2.float() != 0
    frac = kept.float().mean().item()
    assert abs(frac - (1 - p)) < 0.02
    torch.testing.assert_close(s2.float()[kept], torch.full_like(s2.float()[kept], 1 / (1 - p)), rtol=1e-2, atol=1e-2)
    s2.backward(torch.ones_like(s2))
    torch.testing.assert_close(b2.grad.float(), kept.float() / (1 - p), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("shape", [(4, 64, 64), (3, 32, 96), (2, 224, 224)])
@pytest.mark.parametrize("wdtype", [torch.bfloat16, torch.float32])
def test_stem_conv_matches_reference(shape, wdtype):
    """csrc/conv_stem.hip forward + weight gradient vs an fp32 PyTorch conv of the same bf16 data."""
    from determined_amd.ops.conv import stem_conv2d, stem_fusable

    torch.manual_seed(0)
    N, H, W = shape
    conv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).cuda().to(wdtype)
    x = torch.randn(N, 3, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert stem_fusable(conv, x)
    y = stem_conv2d(conv, x)
    xr = x.float()
    wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, stride=2, padding=3)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=3e-2)
    g = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    dw = conv.weight.grad
    assert dw.dtype == wdtype and dw.shape == wr.shape
    rel = ((dw.float() - wr.grad).norm() / wr.grad.norm()).item()
    assert rel < 1e-2, rel


def test_stem_conv_bn_stats_fusion():
    """Stem conv epilogue statistics feed the fused BN+ReLU+MaxPool: same result as the BN
    computing its own statistics."""
    import determined_amd.ops as ops
    from determined_amd.ops.conv import stem_conv2d

    torch.manual_seed(0)
    conv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).cuda().to(torch.bfloat16)
    bn_a, bn_b = ops.BatchNormAct2d(64).cuda(), ops.BatchNormAct2d(64).cuda()
    pool = torch.nn.MaxPool2d(3, 2, 1)
    x = (torch.randn(4, 3, 96, 96, device="cuda") + 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y, part = stem_conv2d(conv, x, with_stats=True)
    assert part is not None and part.shape[1:] == (2, 64)
    out_a = bn_a.forward_maxpool(y, pool, stats_part=part)
    out_b = bn_b.forward_maxpool(y.detach(), pool)
    torch.testing.assert_close(out_a.float(), out_b.float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(bn_a.running_mean, bn_b.running_mean, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(bn_a.running_var, bn_b.running_var, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("shape", [(4, 64, 64), (3, 96, 160), (2, 224, 224)])
@pytest.mark.parametrize("pdtype", [torch.bfloat16, torch.float32])
def test_stem_pool_fused_matches_reference(shape, pdtype):
    """conv_stem.hip stem_pool_* (conv + BN + ReLU + max-pool, no full-size conv output) vs the fp32
    PyTorch composition on the same bf16 data: output, running statistics and the gradients of
    the conv weight and the BN affine parameters, with some BN weights negative (min-pool path)."""
    import determined_amd.ops as ops
    from determined_amd.ops.conv import _StemPoolFn, stem_bn_pool

    torch.manual_seed(0)
    N, H, W = shape
    conv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).cuda().to(pdtype)
    bn = ops.BatchNormAct2d(64).cuda().to(pdtype)
    with torch.no_grad():
        bn.weight.copy_(torch.randn(64) * 0.5 + 0.2)  # ~1/3 negative
        bn.bias.copy_(torch.randn(64) * 0.2)
    pool = torch.nn.MaxPool2d(3, 2, 1)
    x = (torch.randn(N, 3, H, W, device="cuda") + 0.3).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert ops.ext().stem_pool_supported(x, conv.weight)
    rm0, rv0 = bn.running_mean.clone(), bn.running_var.clone()
    y = stem_bn_pool(conv, bn, pool, x)
    assert y.grad_fn is not None and type(y.grad_fn).__name__ == _StemPoolFn.__name__ + "Backward"
    wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    gr = bn.weight.detach().float().requires_grad_(True)
    br = bn.bias.detach().float().requires_grad_(True)
    rmr, rvr = rm0.clone(), rv0.clone()
    c = torch.nn.functional.conv2d(x.float(), wr, stride=2, padding=3)
    c = c + (c.detach().to(torch.bfloat16).float() - c.detach())  # the kernel normalises bf16-rounded outputs
    yr = pool(torch.relu(torch.nn.functional.batch_norm(c, rmr, rvr, gr, br, True, 0.1, bn.eps)))
    assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(bn.running_mean, rmr, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(bn.running_var, rvr, rtol=1e-3, atol=1e-4)
    g = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    for got, ref in ((conv.weight.grad, wr.grad), (bn.weight.grad, gr.grad), (bn.bias.grad, br.grad)):
        assert got.dtype == pdtype
        rel = ((got.float() - ref).norm() / ref.norm()).item()
        assert rel < 2e-2, rel


def test_stem_pool_fused_matches_unfused_kernels():
    """The fused stem against the separate stem conv + BN/ReLU/max-pool kernels it replaces (same
    bf16 arithmetic up to pooling ties and the bf16 sum of the two consumers' gradients)."""
    import determined_amd.ops as ops
    from determined_amd.ops.conv import stem_bn_pool, stem_conv2d

    torch.manual_seed(1)
    conv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).cuda().to(torch.bfloat16)
    bn_a = ops.BatchNormAct2d(64).cuda().to(torch.bfloat16)
    bn_b = ops.BatchNormAct2d(64).cuda().to(torch.bfloat16)
    with torch.no_grad():
        w = torch.randn(64) * 0.5 + 0.3
        bn_a.weight.copy_(w)
        bn_b.weight.copy_(w)
    pool = torch.nn.MaxPool2d(3, 2, 1)
    x = torch.randn(8, 3, 128, 128, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    conv_b = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).cuda().to(torch.bfloat16)
    conv_b.load_state_dict(conv.state_dict())
    ya, ya2 = stem_bn_pool(conv, bn_a, pool, x, split_grad=True)
    yc, part = stem_conv2d(conv_b, x, with_stats=True)
    yb, yb2 = bn_b.forward_maxpool(yc, pool, split_grad=True, stats_part=part)
    torch.testing.assert_close(ya.float(), yb.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(bn_a.running_var, bn_b.running_var, rtol=1e-4, atol=1e-5)
    g1 = torch.randn_like(ya)
    g2 = torch.randn_like(ya)
    ((ya.float() * g1.float()).sum() + (ya2.float() * g2.float()).sum()).backward()
    ((yb.float() * g1.float()).sum() + (yb2.float() * g2.float()).sum()).backward()
    for a, b in ((conv.weight.grad, conv_b.weight.grad), (bn_a.weight.grad, bn_b.weight.grad),
                 (bn_a.bias.grad, bn_b.bias.grad)):
        rel = ((a.float() - b.float()).norm() / b.float().norm()).item()
        assert rel < 1e-2, rel


def test_linear_gelu_fused_matches_reference():
    """Fused GELU forward / GELU'+bias-gradient backward vs the fp32 PyTorch composition."""
    from determined_amd.ops.fused import linear_gelu

    torch.manual_seed(0)
    lin = torch.nn.Linear(256, 1024).cuda().to(torch.bfloat16)
    x = torch.randn(3, 77, 256, device="cuda").to(torch.bfloat16).requires_grad_(True)
    y = linear_gelu(lin, x)
    xr = x.detach().float().requires_grad_(True)
    wr = lin.weight.detach().float().requires_grad_(True)
    br = lin.bias.detach().float().requires_grad_(True)
    yr = torch.nn.functional.gelu(torch.nn.functional.linear(xr, wr, br), approximate="tanh")
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    g = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    for got, ref in ((x.grad, xr.grad), (lin.weight.grad, wr.grad), (lin.bias.grad, br.grad)):
        rel = ((got.float() - ref).norm() / ref.norm()).item()
        assert rel < 1e-2, rel


@pytest.mark.parametrize("shape", [(7, 96), (4096, 1024), (8192, 3072), (3, 5, 4104)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_bias_grad_single_launch(shape, dtype):
    """Column sums with the last-block reduction (csrc/fused.hip): vs fp32 sums, repeated calls
    (the ticket counters must reset themselves) and both output dtypes."""
    import determined_amd.ops as ops

    torch.manual_seed(0)
    g = torch.randn(*shape, device="cuda").to(torch.bfloat16)
    ref = g.float().reshape(-1, shape[-1]).sum(0)
    for _ in range(3):
        out = ops.ext().bias_grad(g, dtype)
        assert out.dtype == dtype and out.shape == (shape[-1],)
        torch.testing.assert_close(out.float(), ref, rtol=1e-2, atol=1e-1)


def test_fused_optimizer_plan_cache_tracks_storage():
    """The cached step plan (fast host path) is rebuilt when a parameter's storage changes."""
    import determined_amd.ops as ops

    p = torch.nn.Parameter(torch.ones(1000, device="cuda"))
    g = torch.ones_like(p)  # one persistent gradient object, as with bucket views
    opt = ops.FusedSGD([p], lr=0.1, momentum=0.0, weight_decay=0.0)
    for _ in range(2):
        p.grad = g
        opt.step()
    torch.testing.assert_close(p.detach(), torch.full_like(p, 0.8))
    p.data = torch.zeros(1000, device="cuda")  # new storage, same Parameter / gradient objects
    p.grad = g
    opt.step()
    torch.testing.assert_close(p.detach(), torch.full_like(p, -0.1))


@pytest.mark.parametrize("cin,cout,k,stride", [(64, 128, 1, 1), (128, 64, 3, 1), (64, 128, 3, 2), (128, 256, 1, 2)])
def test_igemm_conv_autograd_matches_fp32(ops, cin, cout, k, stride):
    """conv_bn_input: forward + BN statistic partials on the implicit-GEMM kernel, input
    gradient (stride 1: flipped-weight forward kernel; tuned against MIOpen), weight gradient."""
    from determined_amd.ops.conv import conv_bn_input

    torch.manual_seed(0)
    conv = torch.nn.Conv2d(cin, cout, k, stride=stride, padding=k // 2, bias=False).cuda().to(torch.bfloat16)
    conv = conv.to(memory_format=torch.channels_last)
    x = torch.randn(4, cin, 14, 14, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y, part = conv_bn_input(conv, x)
    assert "_IGemmConvFn" in type(y.grad_fn).__name__ and part is not None
    xr = x.detach().float().requires_grad_(True)
    wr = conv.weight.detach().float().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, stride=stride, padding=k // 2)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2 * yr.abs().max().item())
    torch.testing.assert_close(part[:, 0].sum(0), yr.detach().sum((0, 2, 3)), rtol=1e-3,
                               atol=2e-3 * yr.detach().abs().sum((0, 2, 3)).max().item())
    dy = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    yr.backward(dy.float())
    assert x.grad.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=2e-2 * xr.grad.abs().max().item())
    torch.testing.assert_close(conv.weight.grad.float(), wr.grad, rtol=2e-2, atol=2e-2 * wr.grad.abs().max().item())


@pytest.mark.parametrize("cin,width,stride", [(64, 64, 1), (256, 64, 1), (256, 128, 2)])
def test_bottleneck_grads_with_and_without_conv_kernels(ops, monkeypatch, cin, width, stride):
    """One ResNet bottleneck (BN statistics from the conv epilogues, split-gradient input pair,
    downsample shortcut when strided) vs the MIOpen composition and vs an fp32 reference.  (Whole
    random-init ResNet-50 gradients are chaotic in bf16 -- every path, the MIOpen one included,
    lands ~100% away from fp32 -- so the comparison is per block.)"""
    from determined_amd.models.resnet import Bottleneck
    from determined_amd.ops.bn import BatchNormAct2d

    torch.manual_seed(0)
    ds = None
    if stride != 1 or cin != 4 * width:
        ds = torch.nn.Sequential(torch.nn.Conv2d(cin, 4 * width, 1, stride=stride, bias=False),
                                 BatchNormAct2d(4 * width, act=False))
    blk = Bottleneck(cin, width, stride, ds)
    for mod in blk.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            torch.nn.init.uniform_(mod.weight, 0.5, 1.5)
    x0 = torch.randn(8, cin, 16, 16)
    g0 = torch.randn(8, 4 * width, 16 // stride, 16 // stride)

    def run(dtype, disabled):
        monkeypatch.setattr(ops, "_DISABLED", frozenset(disabled))
        import copy

        b = copy.deepcopy(blk).cuda().to(dtype).to(memory_format=torch.channels_last)
        x = x0.cuda().to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        y = b((x, x))
        y = y[0] if isinstance(y, tuple) else y
        y.backward(g0.cuda().to(dtype).contiguous(memory_format=torch.channels_last))
        grads = {n: p.grad.float().cpu() for n, p in b.named_parameters()}
        grads["x"] = x.grad.float().cpu()
        return grads

    ref = run(torch.float32, ())
    on = run(torch.bfloat16, ())
    off = run(torch.bfloat16, ("igemm_conv", "conv_stats"))
    for n, r in ref.items():
        e_on = ((on[n] - r).norm() / r.norm()).item()
        e_off = ((off[n] - r).norm() / r.norm()).item()
        assert e_on < max(2 * e_off, 3e-2), (n, e_on, e_off)




@pytest.mark.parametrize("k,masked,with_d2", [(1, True, True), (1, True, False), (3, False, False), (1, False, False)])
def test_conv_dgrad_bn_epilogue(ops, k, masked, with_d2):
    """conv_dgrad_bn: dz = (dX [+ d2]) * relu-mask and the BN-backward partials, vs torch."""
    e = ops.ext()
    torch.manual_seed(0)
    n, cin, cout, hw = 4, 128, 64, 10
    cl = torch.channels_last
    w = (torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5).to(torch.bfloat16)
    g = torch.randn(n, cout, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    yb = torch.randn(n, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    bnw = torch.rand(cin, device="cuda") + 0.5
    bnb = torch.randn(cin, device="cuda") * 0.2
    res = torch.randn_like(yb) if masked else None
    a, stats, mask = e.bn_act_fwd(yb, bnw, bnb, None, None, 0.0, 1e-5, res, True, True, None)
    assert (mask.numel() > 0) == masked
    d2 = torch.randn_like(yb) if with_d2 else None
    wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=cl)
    da = torch.nn.grad.conv2d_input(yb.shape, w.float(), g.float(), padding=k // 2)
    if with_d2:
        da = da + d2.float()
    ref = da * (a.float() > 0)
    cen = yb.float() - stats[0].view(1, -1, 1, 1)
    cfgs = [c for c in range(e.conv_num_cfgs()) if e.conv_supported(g, wt, c, 1, k // 2)]
    assert cfgs
    for cfg in cfgs:  # generic and (3x3) halo kernels
        dz, part = e.conv_dgrad_bn(g, wt, k // 2, cfg, d2, yb, mask if masked else None, stats, None, None)
        torch.testing.assert_close(dz.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
        dzf = dz.float()
        torch.testing.assert_close(part[:, 0].sum(0), dzf.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
        torch.testing.assert_close(part[:, 1].sum(0), (dzf * cen).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("k,hw", [(1, 10), (1, 7), (3, 10)])
def test_conv_dgrad_bn_compact_d2(ops, k, hw):
    """conv_dgrad_bn with d2 on the compact stride-2 grid (the input gradient of a 1x1 stride-2
    shortcut conv, ops/conv.py _StridedGrad) == the same call with d2 materialised at full size."""
    from determined_amd.ops.conv import _StridedGrad

    e = ops.ext()
    torch.manual_seed(5)
    n, cin, cout = 3, 128, 64
    cl = torch.channels_last
    w = (torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5).to(torch.bfloat16)
    wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=cl)
    g = torch.randn(n, cout, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    yb = torch.randn(n, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    res = torch.randn_like(yb)
    _, stats, mask = e.bn_act_fwd(yb, torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2,
                                  None, None, 0.0, 1e-5, res, True, True, None)
    hc = (hw + 1) // 2
    d2c = torch.randn(n, cin, hc, hc, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    d2f = _StridedGrad.materialise(d2c, yb.shape)
    assert torch.equal(d2f[:, :, ::2, ::2], d2c) and d2f[:, :, 1::2].abs().sum().item() == 0
    for cfg in [c for c in range(e.conv_num_cfgs()) if e.conv_supported(g, wt, c, 1, k // 2)]:
        dz_ref, part_ref = e.conv_dgrad_bn(g, wt, k // 2, cfg, d2f, yb, mask, stats, None, None)
        dz, part = e.conv_dgrad_bn(g, wt, k // 2, cfg, d2c, yb, mask, stats, None, None)
        torch.testing.assert_close(dz.float(), dz_ref.float(), rtol=0, atol=0)
        torch.testing.assert_close(part, part_ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("n,k,hw,c", [(16, 2048, 3, 1024), (16, 1024, 6, 512), (16, 512, 12, 256), (2, 2048, 7, 1024)])
def test_conv_1x1_dgrad_every_cfg_small_grids(ops, n, k, hw, c):
    """The stride-1 1x1 input gradient (conv_fwd of dY with the transposed weights) for every tile
    config on the small pixel counts of compact shortcut gradients (M = 144 .. 2304) vs fp32."""
    e = ops.ext()
    torch.manual_seed(2)
    cl = torch.channels_last
    w = (torch.randn(k, c, 1, 1, device="cuda") / k ** 0.5).to(torch.bfloat16)
    wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=cl)
    dy = torch.randn(n, k, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    ref = torch.nn.grad.conv2d_input((n, c, hw, hw), w.float(), dy.float())
    bad = []
    for cfg in [q for q in range(e.conv_num_cfgs()) if e.conv_supported(dy, wt, q, 1, 0)]:
        dx = e.conv_fwd(dy, wt, 1, 0, False, cfg, 0)[0].float()
        err = ((dx - ref).norm() / ref.norm()).item()
        if not err < 1e-2:
            bad.append((cfg, err))
    assert not bad, bad


def test_stage_transition_compact_shortcut_grad(ops, monkeypatch):
    """A chained stage transition (1x1 stride-2 downsample fed by a fused BN->conv node): the
    shortcut's input gradient stays compact and is added in the consumer's dgrad epilogue; the
    gradients match the run with that fusion off and an fp32 reference."""
    import copy
    from determined_amd.models.resnet import Bottleneck, _chain_blocks
    from determined_amd.ops.bn import BatchNormAct2d
    from determined_amd.ops.conv import _StridedGrad

    torch.manual_seed(1)
    ds1 = torch.nn.Sequential(torch.nn.Conv2d(64, 256, 1, bias=False), BatchNormAct2d(256, act=False))
    ds2 = torch.nn.Sequential(torch.nn.Conv2d(256, 512, 1, stride=2, bias=False), BatchNormAct2d(512, act=False))
    blocks = torch.nn.ModuleList([Bottleneck(64, 64, 1, ds1), Bottleneck(256, 128, 2, ds2), Bottleneck(512, 128)])
    for mod in blocks.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            torch.nn.init.uniform_(mod.weight, 0.5, 1.5)
    x0 = torch.randn(8, 64, 16, 16)
    g0 = torch.randn(8, 512, 8, 8)
    seen = []
    orig = _StridedGrad.take.__func__

    def take(cls, g):
        got = orig(cls, g)
        seen.append(got is not None)
        return got

    def run(dtype, disabled):
        monkeypatch.setattr(ops, "_DISABLED", frozenset(disabled))
        bl = copy.deepcopy(blocks).cuda().to(dtype).to(memory_format=torch.channels_last)
        x = x0.cuda().to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        y = _chain_blocks(list(bl), x, False)
        y.backward(g0.cuda().to(dtype).contiguous(memory_format=torch.channels_last))
        grads = {n: p.grad.float().cpu() for n, p in bl.named_parameters()}
        grads["x"] = x.grad.float().cpu()
        return grads

    monkeypatch.setattr(_StridedGrad, "take", classmethod(take))
    ref = run(torch.float32, {"bn_conv"})
    on = run(torch.bfloat16, ())
    assert any(seen) and not _StridedGrad._pending  # the compact gradient was parked and taken
    off = run(torch.bfloat16, {"compact_shortcut_grad"})
    for n, r in ref.items():
        e_on = ((on[n] - r).norm() / r.norm()).item()
        e_off = ((off[n] - r).norm() / r.norm()).item()
        assert e_on < max(1.5 * e_off, 2e-2), (n, e_on, e_off)


@pytest.mark.parametrize("depth", [3])
def test_chained_bottlenecks_match_unchained(ops, monkeypatch, depth):
    """ResNet block chain with every BN fused into its consumer conv's autograd node (ops/conv.py
    bn_act_conv) vs per-block forwards, both against an fp32 reference."""
    import copy
    from determined_amd.models.resnet import Bottleneck, _chain_blocks
    from determined_amd.ops.bn import BatchNormAct2d

    torch.manual_seed(0)
    ds = torch.nn.Sequential(torch.nn.Conv2d(64, 256, 1, bias=False), BatchNormAct2d(256, act=False))
    blocks = torch.nn.ModuleList([Bottleneck(64, 64, 1, ds)] + [Bottleneck(256, 64) for _ in range(depth - 1)])
    for mod in blocks.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            torch.nn.init.uniform_(mod.weight, 0.5, 1.5)
    x0 = torch.randn(8, 64, 16, 16)
    g0 = torch.randn(8, 256, 16, 16)

    def run(dtype, chained):
        monkeypatch.setattr(ops, "_DISABLED", frozenset() if chained else frozenset({"bn_conv"}))
        bl = copy.deepcopy(blocks).cuda().to(dtype).to(memory_format=torch.channels_last)
        x = x0.cuda().to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        if chained:
            y = _chain_blocks(list(bl), x, False)
        else:
            y = x
            for b in bl:
                y = b(y)
        y.backward(g0.cuda().to(dtype).contiguous(memory_format=torch.channels_last))
        grads = {n: p.grad.float().cpu() for n, p in bl.named_parameters()}
        grads["x"] = x.grad.float().cpu()
        return y.detach().float().cpu(), grads

    from determined_amd.ops.conv import _LazyBNGrad

    yr, ref = run(torch.float32, False)
    yc, on = run(torch.bfloat16, True)
    assert not _LazyBNGrad._pending  # every deferred BN backward was taken by its producer
    yu, off = run(torch.bfloat16, False)
    assert ((yc - yr).norm() / yr.norm()).item() < 2e-2
    for n, r in ref.items():
        e_on = ((on[n] - r).norm() / r.norm()).item()
        e_off = ((off[n] - r).norm() / r.norm()).item()
        assert e_on < max(2 * e_off, 3e-2), (n, e_on, e_off)


@pytest.mark.parametrize("with_res", [True, False])
def test_conv_bnact_prologue_matches_composition(ops, with_res):
    """conv_bnact_fwd: BN(+residual)+ReLU applied in the 1x1 conv's operand staging vs bn_act_fwd +
    conv_fwd: a, its mask, z and z's statistics, for every prologue-capable config."""
    e = ops.ext()
    torch.manual_seed(0)
    cl = torch.channels_last
    n, cin, cout, hw = 3, 256, 128, 13  # M = 507: a partial last tile
    y = torch.randn(n, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    res = torch.randn_like(y) if with_res else None
    w = (torch.randn(cout, cin, 1, 1, device="cuda") / cin ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    bnw = torch.rand(cin, device="cuda") + 0.5
    bnb = torch.randn(cin, device="cuda") * 0.2
    a_ref, stats, mask_ref = e.bn_act_fwd(y, bnw, bnb, None, None, 0.0, 1e-5, res, True, True, None)
    z_ref = torch.nn.functional.conv2d(a_ref.float(), w.float())
    cfgs = [c for c in range(e.conv_num_cfgs()) if e.conv_pro_supported(y, w, c)]
    assert cfgs
    for cfg in cfgs:
        z, part, a, mask = e.conv_bnact_fwd(y, w, res, stats, with_res, cfg, None)
        torch.testing.assert_close(a, a_ref, rtol=0, atol=0)
        if with_res:
            assert torch.equal(mask, mask_ref)
        else:
            assert mask.numel() == 0
        torch.testing.assert_close(z.float(), z_ref, rtol=2e-2, atol=2e-2 * z_ref.abs().max().item())
        tol = 2e-3 * z_ref.abs().sum((0, 2, 3)).max().item()
        torch.testing.assert_close(part[:, 0].sum(0), z_ref.sum((0, 2, 3)), rtol=1e-3, atol=tol)


def test_conv_bnact_prologue_folds_residual_bn(ops):
    """conv_bnact_fwd with res_stats: the residual is a BatchNorm's INPUT and that BN's apply is
    folded into the staging too (a = relu(bn(y) + bn_r(y_r))) vs materialising bn_r(y_r) first."""
    e = ops.ext()
    torch.manual_seed(6)
    cl = torch.channels_last
    n, cin, cout, hw = 3, 256, 128, 13
    y = torch.randn(n, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    yr = torch.randn_like(y)
    w = (torch.randn(cout, cin, 1, 1, device="cuda") / cin ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    r, rstats, _ = e.bn_act_fwd(yr, torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2,
                                None, None, 0.0, 1e-5, None, False, True, None)
    bnw, bnb = torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2
    _, stats, _ = e.bn_act_fwd(y, bnw, bnb, None, None, 0.0, 1e-5, None, True, True, None)
    # fp32 reference of the folded form (the materialised r is rounded to bf16 once more)
    a_ref = torch.relu(y.float() * stats[2].view(1, -1, 1, 1) + stats[3].view(1, -1, 1, 1)
                       + yr.float() * rstats[2].view(1, -1, 1, 1) + rstats[3].view(1, -1, 1, 1))
    z_ref = torch.nn.functional.conv2d(a_ref, w.float())
    cfgs = [c for c in range(e.conv_num_cfgs()) if e.conv_pro_supported(y, w, c)]
    assert cfgs
    for cfg in cfgs:
        z, part, a, mask = e.conv_bnact_fwd(y, w, yr, stats, True, cfg, rstats)
        torch.testing.assert_close(a.float(), a_ref, rtol=1e-2, atol=1e-2)
        ref_bits = (a.float() > 0).permute(0, 2, 3, 1).reshape(-1, 8)
        got = torch.stack([(mask.long() >> b) & 1 for b in range(8)], 1).bool()
        assert torch.equal(got, ref_bits)
        torch.testing.assert_close(z.float(), z_ref, rtol=2e-2, atol=2e-2 * z_ref.abs().max().item())


def test_bn_bwd_coef_and_conv_fwd_pro2_match_unfused(ops):
    """Deferred backward of a BN without ReLU (the downsample BN): bn_bwd_coef (reduce + finalize
    only) + conv_fwd_pro2 (1x1 input gradient forming dy = A*dz + B*y + Cc in its staging) vs
    bn_act_bwd's dx followed by the plain input-gradient conv."""
    e = ops.ext()
    torch.manual_seed(8)
    cl = torch.channels_last
    n, k, c, hw = 3, 256, 128, 11
    y = torch.randn(n, k, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    dz = torch.randn_like(y)
    bw = (torch.rand(k, device="cuda") + 0.5)
    _, stats, _ = e.bn_act_fwd(y, bw, torch.randn(k, device="cuda") * 0.2, None, None, 0.0, 1e-5, None, False, True,
                               None)
    dy_ref, dg_ref, db_ref, _ = e.bn_act_bwd(dz, y, None, stats, bw, False, False, None, None)
    coef, dg, db = e.bn_bwd_coef(dz, y, stats, bw)
    torch.testing.assert_close(dg, dg_ref, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db, db_ref, rtol=1e-4, atol=1e-3)
    w = (torch.randn(k, c, 1, 1, device="cuda") / k ** 0.5).to(torch.bfloat16)
    wt = w.transpose(0, 1).contiguous(memory_format=cl)
    dx_ref = torch.nn.grad.conv2d_input((n, c, hw, hw), w.float(), dy_ref.float())
    cfgs = [q for q in range(e.conv_num_cfgs()) if e.conv_pro_supported(dz, wt, q)]
    assert cfgs
    for cfg in cfgs:
        dx, dy = e.conv_fwd_pro2(dz, wt, y, coef, cfg)
        torch.testing.assert_close(dy.float(), dy_ref.float(), rtol=1e-2, atol=1e-2)
        torch.testing.assert_close(dx.float(), dx_ref, rtol=2e-2, atol=2e-2 * dx_ref.abs().max().item())


def test_bn_finalize_part_matches_bn_act_fwd(ops):
    e = ops.ext()
    torch.manual_seed(1)
    y = torch.randn(4, 64, 9, 9, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    yf = y.float()
    part = torch.stack([yf.sum((0, 2, 3)), (yf * yf).sum((0, 2, 3))]).unsqueeze(0).contiguous()
    w = torch.rand(64, device="cuda") + 0.5
    b = torch.randn(64, device="cuda")
    rm1, rv1 = torch.zeros(64, device="cuda"), torch.ones(64, device="cuda")
    rm2, rv2 = rm1.clone(), rv1.clone()
    st = e.bn_finalize_part(part, y.numel() // 64, w, b, rm1, rv1, 0.1, 1e-5)
    _, st_ref, _ = e.bn_act_fwd(y, w, b, rm2, rv2, 0.1, 1e-5, None, True, False, None)
    torch.testing.assert_close(st, st_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rm1, rm2, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rv1, rv2, rtol=1e-4, atol=1e-5)


def test_conv_dgrad_bn_with_deferred_bn_apply(ops):
    """conv_dgrad_bn with pro_y/pro_coef: the operand dy = A*dz + B*y + Cc is formed in the dgrad's
    staging (the next BN's backward apply pass) and returned materialised; dz / partials match
    the kernel run on the explicitly applied dy."""
    e = ops.ext()
    torch.manual_seed(3)
    cl = torch.channels_last
    n, cin, cout, hw = 3, 128, 256, 11
    w = (torch.randn(cout, cin, 1, 1, device="cuda") / cin ** 0.5).to(torch.bfloat16)
    wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=cl)
    dzn = torch.randn(n, cout, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    yn = torch.randn_like(dzn)
    coef = torch.randn(3, cout, device="cuda").contiguous()
    yb = torch.randn(n, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    _, stats, _ = e.bn_act_fwd(yb, torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2,
                               None, None, 0.0, 1e-5, None, True, False, None)
    dy_ref = e.bn_bwd_apply_coef(dzn, yn, coef)
    torch.testing.assert_close(dy_ref.float(), (coef[0].view(1, -1, 1, 1) * dzn.float() + coef[1].view(1, -1, 1, 1)
                                                * yn.float() + coef[2].view(1, -1, 1, 1)), rtol=1e-2, atol=1e-2)
    cfgs = [c for c in range(e.conv_num_cfgs()) if e.conv_pro_supported(dzn, wt, c)]
    assert cfgs
    for cfg in cfgs:
        dz_ref, part_ref = e.conv_dgrad_bn(dy_ref, wt, 0, cfg, None, yb, None, stats, None, None)
        dz, part, dy = e.conv_dgrad_bn(dzn, wt, 0, cfg, None, yb, None, stats, yn, coef)
        torch.testing.assert_close(dy.float(), dy_ref.float(), rtol=1e-2, atol=1e-2)  # fma order may differ by 1 ulp
        torch.testing.assert_close(dz.float(), dz_ref.float(), rtol=1e-2, atol=1e-2)
        torch.testing.assert_close(part, part_ref, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("shape", [(4, 64, 64, 14), (2, 64, 128, 23), (1, 128, 64, 56)])
def test_conv3x3_halo_prologues(ops, shape):
    """3x3 halo kernel with a register-staged prologue: PRO 1 (BN+ReLU forward apply of the input,
    `a` written for the weight gradient) vs bn_act_fwd + conv, and PRO 2 (deferred BN-backward
    apply dy = A*dz + B*y + Cc) vs the kernel run on the explicitly applied dy."""
    e = ops.ext()
    torch.manual_seed(4)
    cl = torch.channels_last
    n, cin, cout, hw = shape
    y = torch.randn(n, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") / (cin * 9) ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    a_ref, stats, _ = e.bn_act_fwd(y, torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2,
                                   None, None, 0.0, 1e-5, None, True, False, None)
    z_ref = torch.nn.functional.conv2d(a_ref.float(), w.float(), padding=1)
    cfgs = [c for c in range(e.conv_num_cfgs()) if e.conv_pro_supported(y, w, c)]
    assert cfgs, "no 3x3 prologue config"
    for cfg in cfgs:
        z, part, a, mask = e.conv_bnact_fwd(y, w, None, stats, False, cfg, None)
        torch.testing.assert_close(a, a_ref, rtol=0, atol=0)
        assert mask.numel() == 0
        torch.testing.assert_close(z.float(), z_ref, rtol=2e-2, atol=2e-2 * z_ref.abs().max().item())
        tol = 2e-3 * z_ref.abs().sum((0, 2, 3)).max().item()
        torch.testing.assert_close(part[:, 0].sum(0), z_ref.sum((0, 2, 3)), rtol=1e-3, atol=tol)
    # PRO 2 on the input gradient (flipped weights): dz of the next BN + its input y -> dy in staging
    wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=cl)  # [cin, cout, 3, 3]
    dzn = torch.randn(n, cout, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    yn = torch.randn_like(dzn)
    coef = torch.randn(3, cout, device="cuda").contiguous()
    yb = torch.randn(n, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    _, stb, _ = e.bn_act_fwd(yb, torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.2,
                             None, None, 0.0, 1e-5, None, True, False, None)
    dy_ref = e.bn_bwd_apply_coef(dzn, yn, coef)
    cfgs = [c for c in range(e.conv_num_cfgs()) if e.conv_pro_supported(dzn, wt, c)]
    assert cfgs
    for cfg in cfgs:
        dz_ref, part_ref = e.conv_dgrad_bn(dy_ref, wt, 1, cfg, None, yb, None, stb, None, None)
        dz, part, dy = e.conv_dgrad_bn(dzn, wt, 1, cfg, None, yb, None, stb, yn, coef)
        torch.testing.assert_close(dy.float(), dy_ref.float(), rtol=1e-2, atol=1e-2)
        torch.testing.assert_close(dz.float(), dz_ref.float(), rtol=1e-2, atol=1e-2)
        torch.testing.assert_close(part, part_ref, rtol=1e-3, atol=1e-2)
        for _ in range(12):  # run-to-run identical (a missing barrier before the first halo
            dz2, _, dy2 = e.conv_dgrad_bn(dzn, wt, 1, cfg, None, yb, None, stb, yn, coef)  # was a race)
            assert torch.equal(dz2, dz) and torch.equal(dy2, dy)


@pytest.mark.parametrize("n,hw", [(3, 21), (2, 56)])
def test_conv1x1_bwd_fused_matches_reference(ops, n, hw):
    """One-pass 1x1 backward (dy formed from a deferred BN backward, input gradient with the
    BN-backward epilogue, weight gradient accumulated in the same pass) vs fp32 references."""
    e = ops.ext()
    torch.manual_seed(6)
    cl = torch.channels_last
    K, C = 256, 64
    yb = torch.randn(n, C, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    a, stats, _ = e.bn_act_fwd(yb, torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.2,
                               None, None, 0.0, 1e-5, None, True, False, None)
    w = (torch.randn(K, C, 1, 1, device="cuda") / C ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    dzn = torch.randn(n, K, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    yn = torch.randn_like(dzn)
    coef = torch.randn(3, K, device="cuda").contiguous()
    assert e.conv1x1_bwd_fused_supported(w)
    dz, part, dw = e.conv1x1_bwd_fused(dzn, yn, coef, w, a, yb, stats)
    dy = e.bn_bwd_apply_coef(dzn, yn, coef).float()
    keep = (yb.float() * stats[2].view(1, -1, 1, 1) + stats[3].view(1, -1, 1, 1)) > 0
    dz_ref = torch.nn.grad.conv2d_input(yb.shape, w.float(), dy) * keep
    torch.testing.assert_close(dz.float(), dz_ref, rtol=2e-2, atol=2e-2 * dz_ref.abs().max().item())
    dzf = dz.float()
    torch.testing.assert_close(part[:, 0].sum(0), dzf.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    cen = yb.float() - stats[0].view(1, -1, 1, 1)
    torch.testing.assert_close(part[:, 1].sum(0), (dzf * cen).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    dw_ref = torch.nn.grad.conv2d_weight(a.float(), w.shape, dy)
    assert dw.shape == w.shape and dw.dtype == w.dtype
    torch.testing.assert_close(dw.float(), dw_ref, rtol=2e-2, atol=2e-2 * dw_ref.abs().max().item())
    dz2, part2, dw2 = e.conv1x1_bwd_fused(dzn, yn, coef, w, a, yb, stats)
    assert torch.equal(dz2, dz) and torch.equal(part2, part) and torch.equal(dw2, dw)
