"""CPU reference path of the fused optimizers must equal torch.optim exactly."""

import pytest
import torch

from determined_amd.ops import FusedAdamW, FusedSGD


def _pair(seed=0):
    torch.manual_seed(seed)
    a = [torch.nn.Parameter(torch.randn(s)) for s in [(5,), (3, 4), (2, 3, 3, 3)]]
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    return a, b


@pytest.mark.parametrize("mode", [True, False])
def test_adam_cpu(mode):
    a, b = _pair()
    oa = FusedAdamW(a, lr=1e-2, weight_decay=0.1, adam_w_mode=mode)
    ob = (torch.optim.AdamW if mode else torch.optim.Adam)(b, lr=1e-2, weight_decay=0.1)
    for _ in range(3):
        for x, y in zip(a, b):
            g = torch.randn_like(x)
            x.grad, y.grad = g.clone(), g.clone()
        oa.step()
        ob.step()
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)


def test_sgd_cpu_with_clip():
    a, b = _pair(1)
    oa = FusedSGD(a, lr=0.1, momentum=0.9, weight_decay=1e-3, nesterov=True)
    oa.set_grad_clipping(0.3)
    ob = torch.optim.SGD(b, lr=0.1, momentum=0.9, weight_decay=1e-3, nesterov=True)
    for _ in range(3):
        for x, y in zip(a, b):
            g = torch.randn_like(x)
            x.grad, y.grad = g.clone(), g.clone()
        torch.nn.utils.clip_grad_norm_(b, 0.3)
        oa.step()
        ob.step()
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)


def test_state_dict_roundtrip():
    a, _ = _pair(2)
    o = FusedAdamW(a, lr=1e-3)
    for x in a:
        x.grad = torch.ones_like(x)
    o.step()
    sd = o.state_dict()
    o2 = FusedAdamW(a, lr=1e-3)
    o2.load_state_dict(sd)
    assert float(o2._step_tensor(torch.device("cpu")).item()) == 1.0
    o2.step()
    assert float(o2._step_tensor(torch.device("cpu")).item()) == 2.0
