"""End-to-end training parity of the fused ResNet-50 path (GPU).

The per-kernel tests compare each HIP kernel with a PyTorch reference on one call; this test
checks the whole composition over several optimizer steps: the bf16 channels-last ResNet-50
with every model-level fusion on (implicit-GEMM convs, BN epilogues / prologues, deferred
BN-backward applies, compact shortcut gradients, stem kernels, fused SGD) must follow the same
loss curve as the same model with all fusions off (PyTorch / MIOpen composition).  A race or a
wrong epilogue in any layer shows up here as a diverging curve (a missing LDS barrier in the 3x3
halo prologue did: its gradients were garbage on some runs only)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

ALL_FUSIONS = frozenset({"stem_conv", "stem_stats", "split_grad", "avgpool", "igemm_conv", "conv_stats", "bn_conv",
                         "bn_prologue", "bn_lazy_bwd", "compact_shortcut_grad", "bn_residual_fold"})


def _curve(disabled, steps, batches, monkeypatch):
    import determined_amd.ops as ops
    from determined_amd.benchmarks.resnet50 import param_groups
    from determined_amd.models.resnet import resnet50

    monkeypatch.setattr(ops, "_DISABLED", disabled)
    torch.manual_seed(0)
    model = resnet50(num_classes=100).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    opt = ops.FusedSGD(param_groups(model, 1e-4), lr=0.02, momentum=0.9, master_weights=True)
    losses = []
    for i in range(steps):
        x, y = batches[i % len(batches)]
        loss = F.cross_entropy(model(x).float(), y)
        loss.backward()
        opt.step()
        model.zero_grad(set_to_none=True)
        losses.append(loss.item())
    return losses


def test_resnet50_fused_training_follows_unfused_curve(monkeypatch):
    import determined_amd.ops as ops

    ops.ext()
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    batches = []
    for _ in range(2):
        x = torch.randn(32, 3, 128, 128, generator=g, device="cuda").to(torch.bfloat16)
        batches.append((x.contiguous(memory_format=torch.channels_last),
                        torch.randint(0, 100, (32,), generator=g, device="cuda")))
    steps = 12
    fused = _curve(frozenset(), steps, batches, monkeypatch)
    plain = _curve(ALL_FUSIONS, steps, batches, monkeypatch)
    fused2 = _curve(frozenset(), steps, batches, monkeypatch)
    assert all(torch.isfinite(torch.tensor(fused)))
    assert fused[-1] < fused[0] and fused[-2] < fused[1], fused  # the two memorised batches both improve
    for i, (a, b) in enumerate(zip(fused, plain)):
        assert abs(a - b) <= 0.05 * abs(b) + 0.02, (i, fused, plain)
    # deterministic kernels: the fused run repeats itself (a race shows up as run-to-run noise)
    for i, (a, b) in enumerate(zip(fused, fused2)):
        assert abs(a - b) <= 1e-2 * abs(b), (i, fused, fused2)  # MIOpen atomics: not bitwise
