"""Data-parallel engine correctness on CPU with gloo (world_size 2)."""

import copy

import torch

from tests.dist_utils import run_distributed


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(
        torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8), torch.nn.ReLU(),
        torch.nn.Flatten(), torch.nn.Linear(8 * 6 * 6, 5),
    )


def _data(rank):
    g = torch.Generator()
    g.manual_seed(100 + rank)
    return torch.randn(4, 3, 8, 8, generator=g)


def _ddp_worker(rank, world, bucket_mb, accumulate):
    from determined_amd.parallel.ddp import DistributedDataParallel

    m = _model().to(memory_format=torch.channels_last)
    ddp = DistributedDataParallel(m, bucket_cap_mb=bucket_mb, first_bucket_mb=bucket_mb)
    out = []
    for it in range(3):
        ddp.zero_grad()
        if accumulate:
            with ddp.no_sync():
                ddp(_data(rank + 10 * it)).sum().backward()
        ddp(_data(rank + 10 * it + 5)).sum().backward()
        ddp.finish()
        out.append({n: p.grad.clone() for n, p in m.named_parameters()})
    return out


def _reference(world, accumulate):
    m = _model().to(memory_format=torch.channels_last)
    res = []
    for it in range(3):
        grads = None
        for r in range(world):
            mm = copy.deepcopy(m)
            mm.zero_grad()
            if accumulate:
                mm(_data(r + 10 * it)).sum().backward()
            mm(_data(r + 10 * it + 5)).sum().backward()
            g = {n: p.grad.clone() for n, p in mm.named_parameters()}
            grads = g if grads is None else {k: grads[k] + g[k] for k in g}
        res.append({k: v / world for k, v in grads.items()})
    return res


def test_ddp_gloo_matches_averaged_grads():
    outs = run_distributed(_ddp_worker, world=2, args=(0.0005, False))
    ref = _reference(2, False)
    for rank_out in outs:
        for it in range(3):
            for k in ref[it]:
                torch.testing.assert_close(rank_out[it][k], ref[it][k], rtol=1e-5, atol=1e-6)


def test_ddp_gloo_no_sync_accumulation():
    outs = run_distributed(_ddp_worker, world=2, args=(1.0, True))
    ref = _reference(2, True)
    for rank_out in outs:
        for it in range(3):
            for k in ref[it]:
                torch.testing.assert_close(rank_out[it][k], ref[it][k], rtol=1e-5, atol=1e-6)


def test_ddp_single_process_grad_views():
    from determined_amd.parallel.ddp import DistributedDataParallel

    m = _model().to(memory_format=torch.channels_last)
    ref = copy.deepcopy(m)
    ddp = DistributedDataParallel(m)
    x = _data(0)
    ddp(x).sum().backward()
    ddp.finish()
    ref(x).sum().backward()
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad, q.grad)
        assert p.grad.stride() == p.stride(), n
    # zero_grad(set_to_none=True) by the user must not break bucket views
    for p in m.parameters():
        p.grad = None
    ddp(x).sum().backward()
    ddp.finish()
    ptrs = {b.buffer.data_ptr() for b in ddp._buckets}
    assert all(any(p.grad.data_ptr() >= bp for bp in ptrs) for p in m.parameters())


def test_ddp_no_sync_before_first_step_keeps_bucket_order_clean():
    """A gradient-less warm-up backward under no_sync (kernel tuning) must not leave its hook order
    behind: the first synced step re-derives the buckets from its own order, each parameter once."""
    import torch

    from determined_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    ddp = DistributedDataParallel(model, bucket_cap_mb=0.0001, first_bucket_mb=0.0001)
    x = torch.randn(5, 8)
    with ddp.no_sync():
        ddp(x).square().sum().backward()
    ddp.zero_grad()
    ddp(x).square().sum().backward()
    ddp.finish()
    ids = [id(p) for b in ddp._buckets for p in b.params]
    assert len(ids) == len(set(ids)) == len(list(model.parameters()))
    ref = torch.nn.Sequential(*[m for m in model])  # same module: grads must equal a plain backward
    g = [p.grad.clone() for p in model.parameters()]
    for p in model.parameters():
        p.grad = None
    ref(x).square().sum().backward()
    for a, b in zip(g, [p.grad for p in model.parameters()]):
        torch.testing.assert_close(a, b)


def test_ddp_tail_bucket_is_small():
    """The last-ready gradients (the first layers) form their own bucket of at most
    ``last_bucket_mb``: its all-reduce is the one that cannot overlap the backward."""
    from determined_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(512, 512), torch.nn.Linear(512, 512), torch.nn.Linear(512, 512),
                            torch.nn.Linear(512, 8))
    mib = 1 << 20
    ddp = DistributedDataParallel(m, bucket_cap_mb=4.0, first_bucket_mb=0.01, last_bucket_mb=1.2)
    sizes = [b.numel * 4 for b in ddp._buckets]
    assert sizes[-1] <= 1.2 * mib and sizes[0] <= 0.02 * mib + 16 * 1024, sizes
    # the tail holds the first layer's parameters (ready last in the backward)
    assert ddp._buckets[-1].params[-1] is m[0].weight or ddp._buckets[-1].params[0] is m[0].bias
    x = torch.randn(4, 512)
    m2 = torch.nn.Sequential(*[torch.nn.Linear(l.in_features, l.out_features) for l in m])
    m2.load_state_dict(m.state_dict())
    ddp(x).square().sum().backward()
    ddp.finish()
    m2(x).square().sum().backward()
    for p, q in zip(m.parameters(), m2.parameters()):
        torch.testing.assert_close(p.grad, q.grad)


def _agree_worker(rank, world):
    import torch

    from determined_amd.ops import conv

    torch.cuda.is_current_stream_capturing = lambda: False  # CPU-only process
    conv._TUNE_ON = True
    # rank 0 alone would fuse (1 < 2); the mean over the ranks (3 vs 2) says no -- on every rank
    t_f = {0: 1.0, 1: 5.0}[rank]
    with conv.agree_across_ranks():
        got = conv._prologue_pays(("agree_test",), lambda: t_f, lambda: 2.0)
        mean = conv._agreed([float(rank), 10.0])
    outside = conv._agreed([float(rank)])
    return torch.tensor([float(got), mean[0], mean[1], outside[0]])


def test_conv_tuning_agrees_across_ranks():
    """Multi-GPU bench tuning (ops/conv.py agree_across_ranks): candidate timings are averaged
    over the ranks, so every rank makes the same kernel choice."""
    outs = run_distributed(_agree_worker, world=2)
    assert outs[0].tolist() == [0.0, 0.5, 10.0, 0.0]
    assert outs[1].tolist() == [0.0, 0.5, 10.0, 1.0]
