"""Flash attention (csrc/attention.hip) with a key-padding mask and in-kernel dropout vs fp32
PyTorch references (GPU).

* key padding: every key a row masks is removed from every query's softmax; forward and all three
  gradients vs fp32 SDPA with the same boolean mask, causal and non-causal, D = 64 / 128, ragged T;
* dropout: with V = identity the output row IS the dropped, rescaled probability row, so the keep
  pattern can be read back; its rate matches p, it is reproducible for a seed, and forward and
  backward agree with an fp32 reference that applies exactly that pattern (the backward recomputes
  the keep decisions from the seed instead of storing them)."""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    import determined_amd.ops as ops

    ops.ext()
    from determined_amd.ops import attention as A

    return A


def _ref(q, k, v, valid=None, causal=False, keep=None, p=0.0):
    s = (q.float() @ k.float().transpose(-1, -2)) / math.sqrt(q.shape[-1])
    T = q.shape[2]
    if causal:
        s = s.masked_fill(torch.ones(T, T, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    if valid is not None:
        s = s.masked_fill(~valid[:, None, None, :], float("-inf"))
    P = torch.softmax(s, -1)
    if keep is not None:
        P = P * keep / (1 - p)
    return P @ v.float()


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("T", [128, 200])
def test_key_padding_mask(D, causal, T):
    A = _ops()
    torch.manual_seed(0)
    B, H = 3, 4
    q, k, v = (torch.randn(B, H, T, D, device="cuda").to(torch.bfloat16).requires_grad_() for _ in range(3))
    lengths = torch.tensor([T, T - 37, 5], device="cuda")
    valid = torch.arange(T, device="cuda")[None, :] < lengths[:, None]
    valid[0, 17] = False  # a hole in the middle, not only right padding
    o = A.flash_attention(q, k, v, causal=causal, key_padding=valid)
    qf, kf, vf = (t.detach().float().requires_grad_() for t in (q, k, v))
    ref = _ref(qf, kf, vf, valid, causal)
    torch.testing.assert_close(o.float(), ref, rtol=2e-2, atol=2e-2)
    do = torch.randn_like(ref)
    o.backward(do.to(torch.bfloat16))
    ref.backward(do)
    for got, want in ((q.grad, qf.grad), (k.grad, kf.grad), (v.grad, vf.grad)):
        torch.testing.assert_close(got.float(), want, rtol=3e-2, atol=3e-2 * want.abs().max().item())
    # padded keys receive no gradient
    assert k.grad[2, :, 5:].abs().max().item() == 0 and v.grad[0, :, 17].abs().max().item() == 0


@pytest.mark.parametrize("D", [64, 128])
def test_dropout_pattern_rate_and_gradients(D):
    A = _ops()
    B, H, T, p = 2, 3, D, 0.25  # T = D so V = identity reads the probability rows back
    torch.manual_seed(1)
    q = (torch.randn(B, H, T, D, device="cuda") * 0.3).to(torch.bfloat16)
    k = (torch.randn(B, H, T, D, device="cuda") * 0.3).to(torch.bfloat16)
    eye = torch.eye(T, D, device="cuda").to(torch.bfloat16).expand(B, H, T, D).contiguous()
    torch.manual_seed(123)
    o1 = A.flash_attention(q, k, eye, causal=False, dropout_p=p)
    torch.manual_seed(123)
    o2 = A.flash_attention(q, k, eye, causal=False, dropout_p=p)
    assert torch.equal(o1, o2)  # same seed -> same pattern
    P = torch.softmax((q.float() @ k.float().transpose(-1, -2)) / math.sqrt(D), -1)
    ratio = o1.float() * (1 - p) / P
    keep = ratio > 0.5
    assert ((ratio[keep] - 1).abs() < 0.05).all() and (ratio[~keep].abs() < 0.05).all()
    rate = 1 - keep.float().mean().item()
    assert abs(rate - p) < 0.03, rate
    # gradients with an arbitrary V under the same seed match the fp32 reference with that pattern
    v = torch.randn(B, H, T, D, device="cuda").to(torch.bfloat16)
    qg, kg, vg = (t.clone().requires_grad_() for t in (q, k, v))
    torch.manual_seed(123)
    o = A.flash_attention(qg, kg, vg, causal=False, dropout_p=p)
    qf, kf, vf = (t.float().requires_grad_() for t in (q, k, v))
    ref = _ref(qf, kf, vf, keep=keep.float(), p=p)
    torch.testing.assert_close(o.float(), ref, rtol=2e-2, atol=2e-2)
    do = torch.randn_like(ref)
    o.backward(do.to(torch.bfloat16))
    ref.backward(do)
    for got, want in ((qg.grad, qf.grad), (kg.grad, kf.grad), (vg.grad, vf.grad)):
        torch.testing.assert_close(got.float(), want, rtol=3e-2, atol=3e-2 * want.abs().max().item())
