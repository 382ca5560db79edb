"""BASELINE config #5 on the GPU: BERT-base masked-LM through the HF Trainer + DetCallback
(examples/hf_bert/run_mlm.py), bf16 with the fused kernels (attention.hip with key padding +
dropout, norm.hip residual-dropout-LayerNorm, fused AdamW) against the stock fp32 model with the
HF AdamW.  Dropout is off for the comparison (the two paths draw different random streams); a
second run with dropout on must stay finite and learn."""

import importlib.util
import pathlib
import tempfile

import pytest

pytestmark = pytest.mark.gpu
transformers = pytest.importorskip("transformers")

ROOT = pathlib.Path(__file__).resolve().parent.parent


def _load_run_mlm():
    spec = importlib.util.spec_from_file_location("run_mlm", ROOT / "examples" / "hf_bert" / "run_mlm.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _train(monkeypatch, extra, steps=8):
    import torch

    from determined_amd import core

    mod = _load_run_mlm()
    losses = []
    with tempfile.TemporaryDirectory() as out, tempfile.TemporaryDirectory() as store:
        margs, targs = mod.parse([
            "--output_dir", out, "--max_steps", str(steps), "--logging_strategy", "steps", "--logging_steps", "1",
            "--eval_strategy", "no", "--save_strategy", "no", "--report_to", "none",
            "--per_device_train_batch_size", "16", "--seq_len", "128", "--train_samples", "4096",
            "--dataloader_num_workers", "0", "--learning_rate", "1e-4", "--warmup_steps", "0",
            "--seed", "0", "--data_seed", "0", *extra])
        torch.manual_seed(0)
        with core.init(checkpoint_storage=store) as ctx:
            monkeypatch.setattr(ctx.train, "report_training_metrics",
                                lambda steps_completed, metrics, **kw: losses.append(metrics.get("loss")))
            mod.main(ctx, margs, targs)
    return [x for x in losses if x is not None]


def test_bert_base_mlm_bf16_fused_follows_fp32(monkeypatch):
    import determined_amd.ops as ops

    ops.ext()
    nodrop = ["--hidden_dropout_prob", "0", "--attention_probs_dropout_prob", "0"]
    fused = _train(monkeypatch, ["--bf16", "true"] + nodrop)
    ref = _train(monkeypatch, ["--stock_kernels", "true", "--hf_optimizer", "true"] + nodrop)
    assert len(fused) == len(ref) == 8, (fused, ref)
    for i, (a, b) in enumerate(zip(fused, ref)):
        assert abs(a - b) <= 0.02 * abs(b) + 0.02, (i, fused, ref)
    assert fused[-1] < fused[0]
    # bf16 parameters with fp32 master weights in the fused AdamW (--bf16_weights)
    bw = _train(monkeypatch, ["--bf16", "true", "--bf16_weights", "true"] + nodrop)
    assert len(bw) == 8
    for i, (a, b) in enumerate(zip(bw, ref)):
        assert abs(a - b) <= 0.03 * abs(b) + 0.03, (i, bw, ref)


def test_bert_base_mlm_with_dropout_trains_like_without(monkeypatch):
    """Dropout on (attention probabilities in attention.hip, hidden states in norm.hip): the loss
    stays finite and within noise of the dropout-free run on the same batches; the fused modules
    really drop (two training-mode forwards differ, eval-mode forwards are identical)."""
    import torch
    import transformers

    from determined_amd.transformers import accelerate

    drop = _train(monkeypatch, ["--bf16", "true"], steps=12)
    nodrop = _train(monkeypatch, ["--bf16", "true", "--hidden_dropout_prob", "0", "--attention_probs_dropout_prob", "0"],
                    steps=12)
    assert len(drop) == len(nodrop) == 12
    assert all(x == x and x < 20 for x in drop)  # finite
    assert abs(sum(drop) / 12 - sum(nodrop) / 12) < 0.15, (drop, nodrop)
    torch.manual_seed(0)
    m = accelerate(transformers.BertForMaskedLM(transformers.BertConfig()).cuda())
    ids = torch.randint(1000, 30000, (4, 128), device="cuda")
    with torch.autocast("cuda", dtype=torch.bfloat16):
        m.train()
        a, b = m(input_ids=ids).logits, m(input_ids=ids).logits
        m.eval()
        c, d = m(input_ids=ids).logits, m(input_ids=ids).logits
    assert not torch.equal(a, b) and torch.equal(c, d)
