"""Tensor parallelism on CPU/gloo: TP=2 GPT-2 matches the dense model (loss, gradients), and
ZeRO over a TP x DP grid matches single-process training including clipped global norms."""

import pytest
import torch

from tests.dist_utils import run_distributed

CFG = dict(n_embd=64, n_layer=2, n_head=4, vocab_size=250, n_positions=32, dropout=0.0, pad_vocab_to=8)


def _dense():
    from determined_amd.models.gpt2 import GPT2Config, GPT2LMHeadModel

    torch.manual_seed(0)
    return GPT2LMHeadModel(GPT2Config(**CFG))


def _tp_worker(rank, world):
    from determined_amd.models.gpt2_tp import GPT2TensorParallel
    from determined_amd.models.gpt2 import GPT2Config
    from determined_amd.parallel import tensor_parallel as tp

    tp.initialize_model_parallel(world)
    dense = _dense()
    model = GPT2TensorParallel(GPT2Config(**CFG))
    model.load_from_dense(dense.state_dict())
    g = torch.Generator().manual_seed(5)
    x = torch.randint(0, 250, (2, 16), generator=g)
    loss = model(x, labels=x)
    loss.backward()
    out = {"loss": loss.detach(), "wpe": model.wpe.weight.grad.clone(),
           "qkv_w": model.h[0].attn.c_attn.weight.grad.clone(), "fc_b": model.h[1].mlp.c_fc.bias.grad.clone(),
           "proj_w": model.h[0].attn.c_proj.weight.grad.clone(), "wte": model.wte.weight.grad.clone(),
           "ln1": model.h[0].ln_1.weight.grad.clone()}
    tp.destroy_model_parallel()
    return out


def test_gpt2_tp2_matches_dense():
    res = run_distributed(_tp_worker, 2)
    dense = _dense()
    g = torch.Generator().manual_seed(5)
    x = torch.randint(0, 250, (2, 16), generator=g)
    loss = dense(x, labels=x)
    loss.backward()
    for r in range(2):
        torch.testing.assert_close(res[r]["loss"], loss.detach(), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(res[r]["wpe"], dense.wpe.weight.grad, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(res[r]["ln1"], dense.h[0].ln_1.weight.grad, rtol=1e-4, atol=1e-5)
    # column-parallel QKV (stride 3): rank r holds rows [blk*C + r*C/2, ...) of each of q, k, v
    C = CFG["n_embd"]
    full = dense.h[0].attn.c_attn.weight.grad
    for r in range(2):
        want = torch.cat([full[b * C + r * C // 2: b * C + (r + 1) * C // 2] for b in range(3)])
        torch.testing.assert_close(res[r]["qkv_w"], want, rtol=1e-4, atol=1e-5)
        half = full.shape[1] // 2
        pw = dense.h[0].attn.c_proj.weight.grad
        torch.testing.assert_close(res[r]["proj_w"], pw[:, r * C // 2:(r + 1) * C // 2], rtol=1e-4, atol=1e-5)
        fb = dense.h[1].mlp.c_fc.bias.grad
        torch.testing.assert_close(res[r]["fc_b"], fb[r * 2 * C:(r + 1) * 2 * C], rtol=1e-4, atol=1e-5)
        del half
    wte = torch.cat([res[0]["wte"], res[1]["wte"]])[:250]
    torch.testing.assert_close(wte, dense.wte.weight.grad[:250], rtol=1e-4, atol=1e-5)


def _grid_worker(rank, world, tp_size, clip):
    from determined_amd.models.gpt2 import GPT2Config
    from determined_amd.models.gpt2_tp import GPT2TensorParallel
    from determined_amd.parallel import tensor_parallel as tp
    from determined_amd.parallel import zero

    tp.initialize_model_parallel(tp_size)
    mpu = tp.get_mpu()
    model = GPT2TensorParallel(GPT2Config(**CFG))
    model.load_from_dense(_dense().state_dict())
    dp = mpu.get_data_parallel_world_size()
    cfg = {"train_micro_batch_size_per_gpu": 2, "gradient_clipping": clip,
           "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.0}},
           "zero_optimization": {"stage": 2, "reduce_bucket_size": 3000}}
    engine, *_ = zero.initialize(model=model, config=cfg, mpu=mpu)
    g = torch.Generator().manual_seed(9)
    for _ in range(3):
        x = torch.randint(0, 250, (2 * dp, 16), generator=g)
        d = mpu.get_data_parallel_rank()
        xs = x[2 * d: 2 * d + 2]
        loss = engine(xs, labels=xs)
        engine.backward(loss)
        engine.step()
    out = {"wpe": model.wpe.weight.detach().clone(), "ln": model.h[1].ln_2.weight.detach().clone(),
           "norm": engine.get_global_grad_norm() if clip > 0 else 0.0}
    tp.destroy_model_parallel()
    return out


@pytest.mark.parametrize("tp_size,world", [(2, 2), (2, 4)])
def test_zero_over_tp_dp_grid_matches_dense(tp_size, world):
    from determined_amd.ops import FusedAdamW

    clip = 0.05
    res = run_distributed(_grid_worker, world, args=(tp_size, clip))
    dense = _dense()
    opt = FusedAdamW(dense.parameters(), lr=1e-2, weight_decay=0.0)
    opt.set_grad_clipping(clip)
    dp = world // tp_size
    g = torch.Generator().manual_seed(9)
    for _ in range(3):
        x = torch.randint(0, 250, (2 * dp, 16), generator=g)
        opt.zero_grad()
        dense(x, labels=x).backward()
        opt.step()
    for r in range(world):
        torch.testing.assert_close(res[r]["wpe"], dense.wpe.weight.detach(), rtol=2e-4, atol=2e-5)
        torch.testing.assert_close(res[r]["ln"], dense.h[1].ln_2.weight.detach(), rtol=2e-4, atol=2e-5)
        assert abs(res[r]["norm"] - float(opt.last_grad_norm)) < 1e-3 * float(opt.last_grad_norm) + 1e-6
