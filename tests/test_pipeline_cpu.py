"""Pipeline parallelism (fill-drain schedule, P2P activations/gradients, ZeRO-1 over each
stage's data-parallel group) on CPU/gloo vs a single-process reference of the same sequential
model (reference tests: DeepSpeed pipeline examples in ``examples/deepspeed/pipeline``)."""

import os
import tempfile

import pytest
import torch
from torch import nn

from tests.dist_utils import run_distributed


def _layers():
    torch.manual_seed(0)
    return [nn.Linear(8, 16), nn.GELU(), nn.Linear(16, 16), nn.LayerNorm(16), nn.Tanh(), nn.Linear(16, 4)]


def _cfg(mb, gas, stage=1):
    return {"train_micro_batch_size_per_gpu": mb, "gradient_accumulation_steps": gas,
            "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.0}},
            "gradient_clipping": 0.0, "zero_optimization": {"stage": stage}}


def _data(steps, n):
    g = torch.Generator().manual_seed(3)
    return [(torch.randn(n, 8, generator=g), torch.randn(n, 4, generator=g)) for _ in range(steps)]


def _loss(out, y):
    return nn.functional.mse_loss(out, y)


def _pipe_worker(rank, world, pp, mb, gas, steps, ckpt):
    from determined_amd.parallel import zero
    from determined_amd.parallel.pipeline import PipelineModule

    dp = world // pp
    module = PipelineModule(_layers(), num_stages=pp, loss_fn=_loss, partition_method="parameters")
    engine, *_ = zero.initialize(model=module, config=_cfg(mb, gas))
    assert engine.is_pipe_parallel and engine.dp == dp
    losses = []
    for x, y in _data(steps, mb * gas * dp):
        # replica d takes micro-batches d, d+dp, ... of the global batch
        d = rank // pp
        mbs = [(x[(k * dp + d) * mb:(k * dp + d + 1) * mb], y[(k * dp + d) * mb:(k * dp + d + 1) * mb])
               for k in range(gas)]
        losses.append(float(engine.train_batch(iter(mbs))))
    ev = float(engine.eval_batch(iter([(x[:mb], y[:mb])]), num_micro_batches=1))
    if ckpt:
        engine.save_checkpoint(ckpt, tag="t")
    sd = {f"{engine.stage_id}.{k}": v.clone() for k, v in engine.module_.state_dict().items()}
    return {"losses": losses, "sd": sd, "parts": module.parts, "eval": ev}


def _reference(dp, mb, gas, steps):
    from determined_amd.ops import FusedAdamW

    m = nn.Sequential(*_layers())
    opt = FusedAdamW(m.parameters(), lr=1e-2, weight_decay=0.0)
    losses = []
    for x, y in _data(steps, mb * gas * dp):
        opt.zero_grad()
        tot = 0.0
        for k in range(gas * dp):
            l = _loss(m(x[k * mb:(k + 1) * mb]), y[k * mb:(k + 1) * mb])
            (l / (gas * dp)).backward()
            tot += float(l)
        opt.step()
        losses.append(tot / (gas * dp))
    return losses, m


@pytest.mark.parametrize("world,pp,gas", [(2, 2, 3), (4, 2, 2)])
def test_pipeline_matches_sequential(world, pp, gas):
    mb, steps = 4, 3
    res = run_distributed(_pipe_worker, world, args=(pp, mb, gas, steps, None))
    ref_losses, ref = _reference(world // pp, mb, gas, steps)
    for r in range(world):
        # every rank returns the (replica-local) loss broadcast from its last stage
        assert len(res[r]["losses"]) == steps
    if world // pp == 1:
        for a, b in zip(res[0]["losses"], ref_losses):
            assert abs(a - b) < 1e-5
    parts = res[0]["parts"]
    merged = {}
    for r in range(pp):  # replica 0's stages
        merged.update(res[r]["sd"])
    ref_sd = ref.state_dict()
    for s in range(pp):
        for li, gi in enumerate(range(parts[s], parts[s + 1])):
            for name in ("weight", "bias"):
                key = f"{gi}.{name}"
                if key in ref_sd:
                    torch.testing.assert_close(merged[f"{s}.layers.{li}.{name}"], ref_sd[key], rtol=2e-5, atol=2e-6)


def test_pipeline_checkpoint_layout():
    with tempfile.TemporaryDirectory() as d:
        run_distributed(_pipe_worker, 2, args=(2, 2, 2, 1, d))
        assert open(os.path.join(d, "latest")).read() == "t"
        for s in range(2):
            assert os.path.exists(os.path.join(d, "t", f"pipe_stage_{s:02d}", "stage", "mp_rank_00_model_states.pt"))


def test_partition_balanced():
    from determined_amd.parallel.pipeline import partition_balanced

    assert partition_balanced([1, 1, 1, 1], 2) == [0, 2, 4]
    assert partition_balanced([10, 1, 1, 10], 2) == [0, 2, 4] or partition_balanced([10, 1, 1, 10], 2) == [0, 1, 4]
    b = partition_balanced([5, 5, 5, 5, 5, 5, 5, 5], 4)
    assert b == [0, 2, 4, 6, 8]
    assert len(partition_balanced([100, 1, 1], 3)) == 4
