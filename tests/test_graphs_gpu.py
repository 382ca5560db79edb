"""Whole-step hipGraph capture (determined_amd.utils.graphs.GraphedStep): a captured training step with
the fused kernels reproduces the eager steps exactly without dropout, and with dropout every replay
draws a fresh pattern from the device-side seeds."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _model():
    transformers = pytest.importorskip("transformers")
    from determined_amd.transformers import accelerate

    cfg = transformers.BertConfig(hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                                  intermediate_size=256, vocab_size=1000, max_position_embeddings=128,
                                  attn_implementation="sdpa")
    torch.manual_seed(0)
    return accelerate(transformers.BertForMaskedLM(cfg).cuda().to(torch.bfloat16))


def _step_fn(model, opt, ids, labels, mask, checksum=False):
    def step():
        out = model(input_ids=ids, attention_mask=mask, labels=labels)
        out.loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
        # (a bf16 loss is too coarse to tell dropout patterns apart: the logits' fp32 checksum is not)
        return out.logits.float().abs().sum() if checksum else out.loss
    return step


def test_graphed_step_matches_eager_without_dropout():
    from determined_amd.ops import FusedAdamW
    from determined_amd.utils.graphs import GraphedStep

    g = torch.Generator(device="cuda").manual_seed(1)
    ids = torch.randint(5, 1000, (4, 64), device="cuda", generator=g)
    labels = torch.where(torch.rand(4, 64, device="cuda", generator=g) < 0.2, ids, torch.full_like(ids, -100))
    mask = torch.ones_like(ids)
    losses = {}
    for mode, n in (("eager", 8), ("graph", 6)):
        model = _model()
        model.eval()  # no dropout anywhere; the optimizer still updates
        opt = FusedAdamW(model.parameters(), lr=1e-3, master_weights=True)
        fn = _step_fn(model, opt, ids, labels, mask)
        step = GraphedStep(fn, warmup=2) if mode == "graph" else fn
        losses[mode] = [float(step()) for _ in range(n)]
    # the graph ran steps 1-2 eagerly as its warm-up; its replays are steps 3-8
    assert losses["graph"] == losses["eager"][2:], losses
    assert losses["eager"][-1] < losses["eager"][0]


def test_graphed_step_redraws_dropout_every_replay():
    from determined_amd.ops import FusedAdamW
    from determined_amd.utils.graphs import GraphedStep

    model = _model()
    model.train()
    opt = FusedAdamW(model.parameters(), lr=0.0, master_weights=True)  # lr 0: the weights stay fixed
    ids = torch.randint(5, 1000, (4, 64), device="cuda")
    labels = ids.clone()
    step = GraphedStep(_step_fn(model, opt, ids, labels, torch.ones_like(ids), checksum=True), warmup=1)
    out = [float(step()) for _ in range(4)]
    assert all(x == x for x in out)
    assert len(set(out)) == 4, out  # fixed weights and inputs: only the dropout pattern changes the logits
