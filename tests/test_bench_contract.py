"""bench.py output contract: one JSON line on stdout with the BASELINE.json metric and config.

The GPU test runs a short single-GPU bench in a child process (batch 64, MIOpen solver search
off so no find-db miss can stall it) and checks every field the round driver reads."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config"}


def test_bench_metric_matches_baseline():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        metric = json.load(f)["metric"]
    with open(os.path.join(ROOT, "bench.py")) as f:
        src = f.read()
    assert json.dumps(metric) in src, "bench.py must report the BASELINE.json metric verbatim"


@pytest.mark.gpu
def test_bench_json_line():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--batch", "64",
                        "--conv-benchmark", "0"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert REQUIRED <= set(out)
    assert out["n_gpus"] == 1 and out["steps"] == 2 and out["warmup"] == 1
    assert out["dtype"] == "bf16" and out["scaling"] == "weak" and out["higher_is_better"] is True
    assert out["config"]["model"] == "resnet50" and out["config"]["global_batch"] == 64
    assert out["value"] > 0 and abs(out["value"] - 64 * 2 / (out["ms_per_step"] * 2 / 1000)) / out["value"] < 0.01
