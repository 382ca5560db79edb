"""ZeRO engine + GPT-2 on the GPU (fused AdamW on shard fragments, bf16 master weights)."""

import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu


def _tiny():
    from determined_amd.models.gpt2 import gpt2

    torch.manual_seed(0)
    return gpt2("gpt2-tiny", dropout=0.0)


def test_gpt2_tiny_forward_backward_matches_fp32():
    m = _tiny().cuda()
    ref = _tiny().double()  # CPU float64 reference
    x = torch.randint(0, 512, (2, 64), device="cuda")
    lo = m(x, labels=x)
    lr = ref(x.cpu(), labels=x.cpu())
    torch.testing.assert_close(lo.double().cpu(), lr, rtol=1e-4, atol=1e-4)
    lo.backward()
    lr.backward()
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad.double().cpu(), q.grad, rtol=1e-3, atol=1e-4, msg=lambda s: f"{n}: {s}")


def test_zero_engine_matches_plain_fused_adamw_bf16():
    """World size 1, stage 2, bf16: the engine's shard update == FusedAdamW(master_weights) on
    the whole model (same kernels; gradient clipping included)."""
    from determined_amd.ops import FusedAdamW
    from determined_amd.parallel import zero

    cfg = {"train_micro_batch_size_per_gpu": 4, "bf16": {"enabled": True}, "gradient_clipping": 0.5,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-3, "weight_decay": 0.1}},
           "zero_optimization": {"stage": 2, "reduce_bucket_size": 20000}}
    engine, *_ = zero.initialize(model=_tiny(), config=cfg)
    ref = _tiny().cuda().bfloat16()
    opt = FusedAdamW(ref.parameters(), lr=1e-3, weight_decay=0.1, master_weights=True)
    opt.set_grad_clipping(0.5)
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(4):
        x = torch.randint(0, 512, (4, 64), device="cuda", generator=g)
        loss = engine(x, labels=x)
        engine.backward(loss)
        engine.step()
        opt.zero_grad()
        ref(x, labels=x).backward()
        opt.step()
    torch.cuda.synchronize()
    sd = engine.module.state_dict()
    for k, v in ref.state_dict().items():
        torch.testing.assert_close(sd[k].float(), v.float(), rtol=2e-2, atol=2e-3, msg=lambda s: f"{k}: {s}")
    assert engine.get_global_grad_norm() is not None


def test_zero_engine_grad_accumulation_fp32_buffer():
    from determined_amd.parallel import zero

    cfg = {"train_micro_batch_size_per_gpu": 2, "gradient_accumulation_steps": 3, "bf16": {"enabled": True},
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}}, "zero_optimization": {"stage": 2}}
    engine, *_ = zero.initialize(model=_tiny(), config=cfg)
    assert engine.spaces[0].G.dtype == torch.float32  # fp32 accumulation across micro-batches
    losses = []
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randint(0, 512, (2, 64), device="cuda", generator=g)
    for _ in range(30):
        loss = engine(x, labels=x)
        engine.backward(loss)
        engine.step()
        losses.append(float(loss))
    assert engine.global_steps == 10
    assert losses[-1] < losses[0] - 0.5


def test_zero3_matches_zero2_bf16_gpu():
    """Stage 3 (partitioned params, per-module gather hooks, tied LM head as an external
    parameter) trains GPT-2 tiny exactly like stage 2 on one GPU with the fused bf16 AdamW."""
    from determined_amd.parallel import zero

    def run(stage):
        cfg = {"train_micro_batch_size_per_gpu": 4, "bf16": {"enabled": True}, "gradient_clipping": 0.0,
               "optimizer": {"type": "AdamW", "params": {"lr": 1e-3, "weight_decay": 0.1}},
               "zero_optimization": {"stage": stage, "reduce_bucket_size": 20000,
                                     "stage3_param_persistence_threshold": 0}}
        engine, *_ = zero.initialize(model=_tiny(), config=cfg)
        g = torch.Generator(device="cuda").manual_seed(0)
        losses = []
        for _ in range(3):
            x = torch.randint(0, 512, (4, 64), device="cuda", generator=g)
            loss = engine(x, labels=x)
            engine.backward(loss)
            engine.step()
            losses.append(float(loss.detach()))
        return losses, engine.state_dict()

    l2, s2 = run(2)
    l3, s3 = run(3)
    assert l2 == l3, (l2, l3)
    for k, v in s2.items():
        torch.testing.assert_close(s3[k], v, rtol=0, atol=0)
