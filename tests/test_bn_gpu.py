"""Fused NHWC BatchNorm(+add)(+ReLU) kernels vs an fp32 PyTorch reference (MI355X)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bnmod():
    import determined_amd.ops as ops

    ops.ext()
    return ops


def _ref(x, w, b, rm, rv, res, relu, mom, eps):
    y = F.batch_norm(x, rm, rv, w, b, True, mom, eps)
    if res is not None:
        y = y + res
    return F.relu(y) if relu else y


@pytest.mark.parametrize("shape", [(4, 64, 14, 14), (2, 256, 7, 9), (3, 2048, 3, 3), (5, 8, 6, 6), (2, 4096, 2, 2)])
@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_act_train(bnmod, shape, res, relu, dtype):
    torch.manual_seed(sum(shape))
    N, C, H, W = shape
    m = bnmod.BatchNormAct2d(C, act=relu).cuda()
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.5, 0.5)
    m = m.to(dtype)
    x = (torch.randn(shape, device="cuda") * 2 + 3).to(dtype).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    r = None
    if res:
        r = torch.randn(shape, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
        r.requires_grad_(True)
    y = m(x, r)
    # fp32 reference
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True) if res else None
    wr = m.weight.detach().float().requires_grad_(True)
    br = m.bias.detach().float().requires_grad_(True)
    rm = torch.zeros(C, device="cuda")
    rv = torch.ones(C, device="cuda")
    yr = _ref(xr, wr, br, rm, rv, rr, relu, 0.1, 1e-5)
    tol = dict(rtol=2e-2, atol=3e-2) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(y.float(), yr, **tol)
    torch.testing.assert_close(m.running_mean, rm, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(m.running_var, rv, rtol=1e-3, atol=1e-3)
    gy = torch.randn_like(yr)
    (y.float() * gy).sum().backward()
    (yr * gy).sum().backward()
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)
    gtol = dict(rtol=3e-2, atol=3e-1) if dtype == torch.bfloat16 else dict(rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(m.weight.grad.float(), wr.grad, **gtol)
    torch.testing.assert_close(m.bias.grad.float(), br.grad, **gtol)
    if res:
        torch.testing.assert_close(r.grad.float(), rr.grad, **tol)


def test_bn_large_mean_stats_stable(bnmod):
    # |mean| >> std: shifted-sum statistics must not cancel.
    C = 64
    m = bnmod.BatchNormAct2d(C, act=False).cuda()
    x = (torch.randn(8, C, 32, 32, device="cuda") * 0.01 + 100.0).contiguous(memory_format=torch.channels_last)
    y = m(x)
    # float64 CPU reference (a single-pass fp32 E[x^2]-E[x]^2 reference would itself cancel here)
    xd = x.detach().double().cpu()
    yr = F.batch_norm(xd, None, None, m.weight.double().cpu(), m.bias.double().cpu(), True, 0.1, 1e-5)
    torch.testing.assert_close(y.double().cpu(), yr, rtol=1e-3, atol=5e-3)


def test_bn_eval_matches(bnmod):
    C = 256
    m = bnmod.BatchNormAct2d(C).cuda()
    with torch.no_grad():
        m.running_mean.uniform_(-1, 1)
        m.running_var.uniform_(0.5, 2)
        m.weight.uniform_(0.5, 1.5)
    m.eval()
    x = torch.randn(2, C, 5, 5, device="cuda").contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x)
    with torch.no_grad():
        y = m(x, r)
    yr = F.relu(F.batch_norm(x, m.running_mean, m.running_var, m.weight, m.bias, False, 0.1, 1e-5) + r)
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)


def test_bf16_model_keeps_fp32_running_stats(bnmod):
    m = bnmod.BatchNormAct2d(64).cuda().to(torch.bfloat16)
    assert m.running_mean.dtype == torch.float32 and m.weight.dtype == torch.bfloat16


@pytest.mark.parametrize("shape", [(4, 64, 112, 112), (3, 16, 13, 10), (2, 8, 7, 8)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_relu_maxpool_fused_matches_reference(bnmod, shape, dtype):
    """ResNet stem: fused BN+ReLU+MaxPool(3,2,1) fwd/bwd vs the fp32 PyTorch composition."""
    torch.manual_seed(0)
    N, C, H, W = shape
    m = bnmod.BatchNormAct2d(C).cuda()
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.5, 0.5)
    pool = torch.nn.MaxPool2d(3, 2, 1)
    x = torch.randn(N, C, H, W, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = m.forward_maxpool(x, pool)
    ref_bn = torch.nn.BatchNorm2d(C).cuda()
    ref_bn.load_state_dict({k: v for k, v in m.state_dict().items()}, strict=False)
    with torch.no_grad():
        ref_bn.weight.copy_(m.weight.float())
        ref_bn.bias.copy_(m.bias.float())
        ref_bn.running_mean.zero_()
        ref_bn.running_var.fill_(1.0)
    xr = x.detach().float().requires_grad_(True)
    yr = pool(torch.relu(ref_bn(xr)))
    tol = dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(y.float(), yr, **tol)
    assert y.is_contiguous(memory_format=torch.channels_last) and y.shape == yr.shape
    g = torch.randn_like(yr).to(dtype)  # both sides get the same (dtype-rounded) upstream gradient
    y.backward(g)
    yr.backward(g.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, **tol)
    torch.testing.assert_close(m.weight.grad.float(), ref_bn.weight.grad, rtol=2e-2, atol=5e-2)
    torch.testing.assert_close(m.bias.grad.float(), ref_bn.bias.grad, rtol=2e-2, atol=5e-2)
    torch.testing.assert_close(m.running_mean, ref_bn.running_mean, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_split_grad_sums_both_consumers(bnmod, dtype):
    """split_grad: the two handles' gradients are summed inside the BN backward kernels (block
    output feeding conv + shortcut) -- same result as autograd's accumulation of one output."""
    torch.manual_seed(0)
    N, C, H, W = 4, 64, 14, 14
    m = bnmod.BatchNormAct2d(C).cuda()
    mk = lambda: torch.randn(N, C, H, W, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    x, res, g1, g2 = mk(), mk(), mk(), mk()
    xa = x.clone().requires_grad_(True)
    ra = res.clone().requires_grad_(True)
    ya, yb = m(xa, ra, split_grad=True)
    assert ya.data_ptr() == yb.data_ptr()
    (ya * g1.float()).sum().backward(retain_graph=True)
    (yb * g2.float()).sum().backward()
    dga, dba = m.weight.grad.clone(), m.bias.grad.clone()
    m.zero_grad()
    xr = x.clone().requires_grad_(True)
    rr = res.clone().requires_grad_(True)
    y = m(xr, rr)
    y.backward(g1 + g2 if dtype == torch.float32 else (g1.float() + g2.float()).to(dtype))
    tol = dict(rtol=2e-2, atol=3e-2) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(xa.grad.float(), xr.grad.float(), **tol)
    torch.testing.assert_close(ra.grad.float(), rr.grad.float(), **tol)
    # dgamma/dbeta sum ~800 terms (|sum| ~ 40): the unsplit side rounds g1 + g2 to bf16 per
    # element first, the split side sums in fp32, so bf16 allows that accumulated rounding
    ptol = dict(rtol=2e-2, atol=2.5e-1) if dtype == torch.bfloat16 else dict(rtol=2e-2, atol=5e-2)
    torch.testing.assert_close(dga.float(), m.weight.grad.float(), **ptol)
    torch.testing.assert_close(dba.float(), m.bias.grad.float(), **ptol)


def test_resnet_split_grad_chain_matches_unsplit(bnmod):
    """ResNet-50 with split-gradient block chaining vs the plain Sequential chain.  MIOpen's
    convolutions are not bitwise reproducible run to run (atomic weight gradients), so the
    plain chain is run twice and that noise floor bounds the split-vs-plain difference."""
    from determined_amd.models.resnet import resnet50

    torch.manual_seed(0)
    model = resnet50(num_classes=10, zero_init_residual=False).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 128, 128, device="cuda").contiguous(memory_format=torch.channels_last)
    state = {k: v.clone() for k, v in model.state_dict().items()}

    def plain(inp):
        h = model.bn1.forward_maxpool(model.conv1(inp), model.maxpool)
        h = model.layer4(model.layer3(model.layer2(model.layer1(h))))
        return model.fc(torch.flatten(model.avgpool(h), 1))

    def grads(fn):
        model.load_state_dict(state)
        model.zero_grad()
        fn(x).float().square().mean().backward()
        return {n: p.grad.clone() for n, p in model.named_parameters()}

    ref, ref2, split = grads(plain), grads(plain), grads(model)
    rel = lambda a, b: ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
    noise = max(rel(ref2[n], ref[n]) for n in ref)
    worst = max(rel(split[n], ref[n]) for n in ref)
    assert worst <= max(3 * noise, 1e-3), (worst, noise)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_global_avg_pool_bwd(bnmod, dtype):
    """channels-last global average pool: fused broadcast backward vs adaptive_avg_pool2d."""
    from determined_amd.ops.bn import global_avg_pool

    x = torch.randn(6, 2048, 7, 5, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    xa = x.clone().requires_grad_(True)
    xr = x.float().requires_grad_(True)
    ya = global_avg_pool(xa)
    yr = torch.flatten(F.adaptive_avg_pool2d(xr, 1), 1)
    tol = dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ya.float(), yr, **tol)
    g = torch.randn_like(yr).to(dtype)
    ya.backward(g)
    yr.backward(g.float())
    assert xa.grad.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(xa.grad.float(), xr.grad, **tol)


def test_resnet50_bf16_fused_gradients_match_unfused(bnmod, monkeypatch):
    """bf16 channels-last ResNet-50 through every fused path (implicit-GEMM convs, BN epilogues /
    prologues, deferred BN-backward apply, split gradients, stem kernels) vs the same model with
    all model-level fusions switched off (PyTorch/MIOpen composition).  Both are compared with an
    fp32 run of the same weights: the fused error may not exceed the unfused bf16 error by more
    than a small margin, per parameter."""
    import determined_amd.ops as ops
    from determined_amd.models.resnet import resnet50

    all_fusions = frozenset({"stem_conv", "stem_stats", "split_grad", "avgpool", "igemm_conv", "conv_stats",
                             "bn_conv", "bn_prologue", "bn_lazy_bwd", "compact_shortcut_grad", "bn_residual_fold"})
    torch.manual_seed(0)
    model = resnet50(num_classes=10, zero_init_residual=False).cuda().to(memory_format=torch.channels_last)
    state = {k: v.clone() for k, v in model.state_dict().items()}
    x = torch.randn(16, 3, 96, 96, device="cuda").contiguous(memory_format=torch.channels_last)

    def grads(dtype, disabled):
        monkeypatch.setattr(ops, "_DISABLED", disabled)
        model.load_state_dict(state)
        model.to(dtype)
        model.zero_grad()
        model(x.to(dtype)).float().square().mean().backward()
        out = {n: p.grad.float().clone() for n, p in model.named_parameters()}
        model.float()
        return out

    ref = grads(torch.float32, all_fusions)
    fused = grads(torch.bfloat16, frozenset())
    plain = grads(torch.bfloat16, all_fusions)
    rel = lambda a, b: ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
    for n in ref:
        ef, ep = rel(fused[n], ref[n]), rel(plain[n], ref[n])
        assert ef <= 1.5 * ep + 2e-2, (n, ef, ep)
