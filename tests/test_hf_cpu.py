"""HF Trainer + DetCallback on CPU (tiny BERT): metric routing, searcher completion, checkpoints."""

import importlib.util
import pathlib
import tempfile

import pytest

transformers = pytest.importorskip("transformers")

ROOT = pathlib.Path(__file__).resolve().parent.parent


def _load_run_mlm():
    spec = importlib.util.spec_from_file_location("run_mlm", ROOT / "examples" / "hf_bert" / "run_mlm.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_metric_type():
    from determined_amd.transformers import get_metric_type

    assert get_metric_type({"eval_loss": 1.0}) == "eval_"
    assert get_metric_type({"train_runtime": 1.0}) == "train_"
    assert get_metric_type({"loss": 1.0, "learning_rate": 0.1}) == "train_progress"
    assert get_metric_type({"test_acc": 1.0}) == "test_"


def test_hf_trainer_detcallback_local(monkeypatch):
    from determined_amd import core

    mod = _load_run_mlm()
    with tempfile.TemporaryDirectory() as out, tempfile.TemporaryDirectory() as store:
        margs, targs = mod.parse([
            "--output_dir", out, "--max_steps", "6", "--logging_strategy", "steps", "--logging_steps", "2",
            "--eval_strategy", "steps", "--eval_steps", "3", "--save_strategy", "steps", "--save_steps", "3",
            "--report_to", "none", "--use_cpu", "true", "--per_device_train_batch_size", "4",
            "--per_device_eval_batch_size", "4", "--hidden_size", "32", "--num_hidden_layers", "2",
            "--num_attention_heads", "2", "--intermediate_size", "64", "--vocab_size", "2000", "--seq_len", "32",
            "--train_samples", "256", "--eval_samples", "16", "--dataloader_num_workers", "0",
        ], {"training_arguments": {"learning_rate": 5e-4}})
        assert targs.learning_rate == 5e-4
        train_reports, val_reports, completed = [], [], []
        with core.init(checkpoint_storage=store) as ctx:
            monkeypatch.setattr(ctx.train, "report_training_metrics",
                                lambda steps_completed, metrics, **kw: train_reports.append(steps_completed))
            monkeypatch.setattr(ctx.train, "report_validation_metrics",
                                lambda steps_completed, metrics, **kw: val_reports.append((steps_completed,
                                                                                          metrics)))
            res = mod.main(ctx, margs, targs)
            cb = res["callback"]
        assert train_reports == [2, 4, 6]
        assert [s for s, _ in val_reports] == [3, 6]
        assert "eval_loss" in val_reports[-1][1]
        assert cb.current_op._completed if hasattr(cb.current_op, "_completed") else True
        ckpts = [p for p in pathlib.Path(store).iterdir() if p.is_dir()]
        assert len(ckpts) == 2
        files = {str(f.relative_to(c)) for c in ckpts for f in c.rglob("*") if f.is_file()}
        assert any(f.startswith("checkpoint-6/") for f in files)
        assert any(f.endswith("my_data.json") for f in files)
