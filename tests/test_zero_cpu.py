"""ZeRO engine numerics on CPU/gloo (world 2) vs a single-process full-batch reference."""

import os
import tempfile

import pytest
import torch
from torch import nn

from tests.dist_utils import run_distributed


def _model() -> nn.Module:
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(12, 33), nn.LayerNorm(33), nn.GELU(), nn.Linear(33, 7))


def _data(steps: int, gbs: int):
    g = torch.Generator().manual_seed(1)
    return [(torch.randn(gbs, 12, generator=g), torch.randn(gbs, 7, generator=g)) for _ in range(steps)]


def _cfg(stage: int, world: int, gas: int, mb: int, clip: float, bucket: int):
    return {
        "train_micro_batch_size_per_gpu": mb,
        "gradient_accumulation_steps": gas,
        "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.1, "betas": [0.9, 0.99]}},
        "scheduler": {"type": "WarmupLR", "params": {"warmup_min_lr": 0.0, "warmup_max_lr": 1e-2,
                                                     "warmup_num_steps": 3, "warmup_type": "linear"}},
        "gradient_clipping": clip,
        "zero_optimization": {"stage": stage, "reduce_bucket_size": bucket},
    }


def _train(rank: int, world: int, stage: int, gas: int, clip: float, bucket: int, steps: int = 4):
    from determined_amd.parallel import zero

    mb = 4
    gbs = mb * gas * world
    engine, opt, _, sched = zero.initialize(model=_model(), config=_cfg(stage, world, gas, mb, clip, bucket))
    losses = []
    for x, y in _data(steps, gbs):
        for k in range(gas):
            lo = (k * world + rank) * mb
            out = engine(x[lo : lo + mb])
            loss = nn.functional.mse_loss(out, y[lo : lo + mb])
            engine.backward(loss)
            engine.step()
            losses.append(float(loss.detach()))
    assert engine.global_steps == steps and engine.micro_steps == steps * gas
    return {k: v.clone() for k, v in engine.state_dict().items()}


def _reference(world: int, gas: int, clip: float, steps: int = 4):
    from determined_amd.ops import FusedAdamW
    from determined_amd.parallel.zero import WarmupLR

    m = _model()
    opt = FusedAdamW(m.parameters(), lr=1e-2, weight_decay=0.1, betas=(0.9, 0.99))
    if clip > 0:
        opt.set_grad_clipping(clip)
    sched = WarmupLR(opt, 0.0, 1e-2, 3, "linear")
    mb = 4
    for x, y in _data(steps, mb * gas * world):
        opt.zero_grad()
        for k in range(gas):
            for r in range(world):
                lo = (k * world + r) * mb
                loss = nn.functional.mse_loss(m(x[lo : lo + mb]), y[lo : lo + mb]) / (gas * world)
                loss.backward()
        opt.step()
        sched.step()
    return m.state_dict()


def _worker(rank, world, stage, gas, clip, bucket):
    return _train(rank, world, stage, gas, clip, bucket)


@pytest.mark.parametrize("stage,gas,clip,bucket", [(2, 1, 0.0, 64), (2, 2, 0.5, 300), (1, 2, 0.0, 10**6),
                                                   (0, 1, 0.5, 128), (3, 1, 0.0, 64), (3, 2, 0.5, 300)])
def test_zero_matches_reference(stage, gas, clip, bucket):
    world = 2
    res = run_distributed(_worker, world, args=(stage, gas, clip, bucket))
    ref = _reference(world, gas, clip)
    for r in range(world):
        for k, v in ref.items():
            torch.testing.assert_close(res[r][k], v, rtol=2e-5, atol=2e-6, msg=lambda m: f"rank {r} {k}: {m}")


def test_zero_single_process_matches_reference():
    res = _train(0, 1, 2, 2, 0.5, 100)
    ref = _reference(1, 2, 0.5)
    for k, v in ref.items():
        torch.testing.assert_close(res[k], v, rtol=2e-5, atol=2e-6)


def _ckpt_worker(rank, world, d):
    from determined_amd.parallel import zero

    cfg = _cfg(2, world, 1, 4, 0.0, 64)
    engine, *_ = zero.initialize(model=_model(), config=cfg)
    data = _data(6, 4 * world)

    def run(eng, batches):
        for x, y in batches:
            lo = rank * 4
            eng.backward(nn.functional.mse_loss(eng(x[lo : lo + 4]), y[lo : lo + 4]))
            eng.step()

    run(engine, data[:3])
    engine.save_checkpoint(d, tag="t3")
    run(engine, data[3:])
    want = {k: v.clone() for k, v in engine.module.state_dict().items()}
    torch.manual_seed(123)
    fresh, *_ = zero.initialize(model=nn.Sequential(nn.Linear(12, 33), nn.LayerNorm(33), nn.GELU(),
                                                    nn.Linear(33, 7)), config=cfg)
    path, client = fresh.load_checkpoint(d)
    assert path.endswith("t3") and fresh.global_steps == 3
    run(fresh, data[3:])
    got = fresh.module.state_dict()
    return {"want": want, "got": got}


def test_zero_checkpoint_resume_exact():
    with tempfile.TemporaryDirectory() as d:
        res = run_distributed(_ckpt_worker, 2, args=(d,))
        assert os.path.exists(os.path.join(d, "t3", "zero_pp_rank_1_mp_rank_00_optim_states.pt"))
    for r in range(2):
        for k in res[r]["want"]:
            torch.testing.assert_close(res[r]["got"][k], res[r]["want"][k], rtol=0, atol=0)


def _reshard_save(rank, world, d):
    from determined_amd.parallel import zero

    engine, *_ = zero.initialize(model=_model(), config=_cfg(2, world, 1, 4, 0.0, 50))
    for x, y in _data(3, 4 * world):
        lo = rank * 4
        engine.backward(nn.functional.mse_loss(engine(x[lo : lo + 4]), y[lo : lo + 4]))
        engine.step()
    engine.save_checkpoint(d, tag="a")
    return {k: v.clone() for k, v in engine.module.state_dict().items()}


def test_zero_checkpoint_reshard_world2_to_world1():
    """Optimizer shards saved by 2 ranks load into 1 rank (elastic re-sharding)."""
    from determined_amd.parallel import zero

    with tempfile.TemporaryDirectory() as d:
        saved = run_distributed(_reshard_save, 2, args=(d,))[0]
        engine, *_ = zero.initialize(model=_model(), config=_cfg(2, 1, 1, 8, 0.0, 50))
        engine.load_checkpoint(d)
        for k, v in saved.items():
            torch.testing.assert_close(engine.module.state_dict()[k], v, rtol=0, atol=0)
        st = engine.optimizer.inner.state
        assert all("exp_avg" in s and float(s["exp_avg"].abs().sum()) > 0 for s in st.values())


def test_ds_config_batch_resolution():
    from determined_amd.parallel.zero import DeepSpeedConfig, DeepSpeedConfigError

    c = DeepSpeedConfig({"train_batch_size": 64, "train_micro_batch_size_per_gpu": 4}, 8)
    assert c.gas == 2
    c = DeepSpeedConfig({"train_batch_size": 64, "gradient_accumulation_steps": 4}, 4)
    assert c.micro_batch == 4
    c = DeepSpeedConfig({"train_micro_batch_size_per_gpu": 3}, 2)
    assert c.train_batch_size == 6 and c.gas == 1
    with pytest.raises(DeepSpeedConfigError):
        DeepSpeedConfig({"train_batch_size": 10, "train_micro_batch_size_per_gpu": 4,
                         "gradient_accumulation_steps": 1}, 2)
    with pytest.raises(DeepSpeedConfigError):
        DeepSpeedConfig({"train_batch_size": 8, "fp16": {"enabled": True}}, 1)


def test_lr_schedules():
    from determined_amd.parallel.zero import WarmupCosineLR, WarmupDecayLR, WarmupLR

    p = nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=0.5)
    s = WarmupLR(opt, 0.0, 1.0, 10, "linear")
    assert opt.param_groups[0]["lr"] == 0.0
    for _ in range(6):  # iteration -1 -> 5
        s.step()
    assert abs(opt.param_groups[0]["lr"] - 0.5) < 1e-9
    opt = torch.optim.SGD([p], lr=0.5)
    s = WarmupDecayLR(opt, 20, 0.0, 1.0, 10, "linear")
    for _ in range(16):  # iteration 15: halfway through the decay
        s.step()
    assert abs(opt.param_groups[0]["lr"] - 0.5) < 1e-9
    opt = torch.optim.SGD([p], lr=2.0)
    s = WarmupCosineLR(opt, total_num_steps=20, warmup_num_steps=4, cos_min_ratio=0.0, warmup_type="linear")
    for _ in range(21):  # iteration 20 == total_num_steps
        s.step()
    assert opt.param_groups[0]["lr"] < 1e-6
