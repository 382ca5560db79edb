"""MFMA flash attention (csrc/attention.hip) vs an fp32 PyTorch reference of the same op."""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(q, k, v, causal):
    qf, kf, vf = q.float(), k.float(), v.float()
    s = qf @ kf.transpose(-1, -2) / math.sqrt(q.shape[-1])
    if causal:
        T = q.shape[2]
        s = s.masked_fill(torch.ones(T, T, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    return torch.softmax(s, -1) @ vf, torch.logsumexp(s, -1)


SHAPES = [(2, 3, 64, 64), (1, 2, 100, 64), (2, 2, 257, 128), (1, 4, 512, 64), (1, 1, 33, 128)]


@pytest.mark.parametrize("B,H,T,D", SHAPES)
@pytest.mark.parametrize("causal", [True, False])
def test_flash_forward(B, H, T, D, causal):
    from determined_amd import ops

    torch.manual_seed(0)
    q, k, v = (torch.randn(B, H, T, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    o, lse = ops.ext().attn_fwd(q, k, v, causal, 1.0 / math.sqrt(D))
    ro, rlse = _ref(q, k, v, causal)
    torch.testing.assert_close(o.float(), ro, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(lse, rlse, rtol=1e-3, atol=2e-3)


@pytest.mark.parametrize("B,H,T,D", SHAPES)
@pytest.mark.parametrize("causal", [True, False])
def test_flash_backward(B, H, T, D, causal):
    from determined_amd.ops.attention import flash_attention

    torch.manual_seed(1)
    base = [torch.randn(B, H, T, D, device="cuda", dtype=torch.bfloat16) for _ in range(3)]
    q, k, v = (t.clone().requires_grad_(True) for t in base)
    o = flash_attention(q, k, v, causal=causal)
    do = torch.randn_like(o)
    o.backward(do)
    rq, rk, rv = (t.float().clone().requires_grad_(True) for t in base)
    ro, _ = _ref(rq, rk, rv, causal)
    ro.backward(do.float())
    for got, want, name in ((q.grad, rq.grad, "dq"), (k.grad, rk.grad, "dk"), (v.grad, rv.grad, "dv")):
        err = (got.float() - want).abs().max().item()
        scale = want.abs().max().item()
        assert err <= 2e-2 * scale + 2e-2, f"{name}: max err {err} (ref max {scale})"


def test_qkv_packed_matches_unpacked():
    from determined_amd.ops.attention import flash_attention, qkv_attention

    torch.manual_seed(2)
    B, T, H, D = 2, 192, 4, 64
    qkv = torch.randn(B, T, 3, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    o = qkv_attention(qkv)
    assert o.shape == (B, H, T, D) and o.transpose(1, 2).is_contiguous()
    do = torch.randn_like(o)
    o.backward(do)
    q2 = qkv.detach().clone().requires_grad_(True)
    q, k, v = q2.permute(2, 0, 3, 1, 4).unbind(0)
    o2 = flash_attention(q, k, v)
    o2.backward(do)
    torch.testing.assert_close(o, o2, rtol=0, atol=0)
    torch.testing.assert_close(qkv.grad, q2.grad, rtol=0, atol=0)


def test_gpt2_block_uses_kernel():
    from determined_amd.models.gpt2 import gpt2

    torch.manual_seed(0)
    m = gpt2("gpt2-tiny", dropout=0.0).cuda().bfloat16()
    x = torch.randint(0, 512, (2, 128), device="cuda")
    loss = m(x, labels=x)
    loss.backward()
    assert torch.isfinite(loss) and all(torch.isfinite(p.grad).all() for p in m.parameters())


@pytest.mark.parametrize("V,Vp", [(50257, 50304), (512, 512), (1000, 1008)])
def test_lm_cross_entropy_matches_reference(V, Vp):
    from determined_amd.ops.fused import lm_cross_entropy

    torch.manual_seed(3)
    B, T = 2, 37
    base = (torch.randn(B, T, Vp, device="cuda") * 3).bfloat16()
    labels = torch.randint(0, V, (B, T), device="cuda")
    labels[0, 5] = -100
    lg = base.clone().requires_grad_(True)
    loss = lm_cross_entropy(lg, labels, V)
    loss.backward()
    ref = base.float().clone().requires_grad_(True)
    rl = torch.nn.functional.cross_entropy(ref[:, :-1, :V].reshape(-1, V), labels[:, 1:].reshape(-1),
                                           ignore_index=-100)
    rl.backward()
    torch.testing.assert_close(loss.float(), rl, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(lg.grad.float(), ref.grad, rtol=2e-2, atol=1e-4)


def test_fused_linear_bias_grad():
    from determined_amd.ops.fused import FusedLinear

    torch.manual_seed(4)
    lin = FusedLinear(64, 96).cuda().bfloat16()
    ref = torch.nn.Linear(64, 96).cuda().float()
    ref.load_state_dict({k: v.float() for k, v in lin.state_dict().items()})
    x = torch.randn(4, 33, 64, device="cuda").bfloat16()
    xr = x.float().requires_grad_(True)
    xb = x.clone().requires_grad_(True)
    dy = torch.randn(4, 33, 96, device="cuda").bfloat16()
    lin(xb).backward(dy)
    ref(xr).backward(dy.float())
    torch.testing.assert_close(lin.bias.grad.float(), ref.bias.grad, rtol=1e-2, atol=5e-2)
    torch.testing.assert_close(lin.weight.grad.float(), ref.weight.grad, rtol=2e-2, atol=1e-1)
    torch.testing.assert_close(xb.grad.float(), xr.grad, rtol=2e-2, atol=5e-2)
