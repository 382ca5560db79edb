"""Data-parallel training of the fused ResNet-50 on one GPU with 2 gloo ranks (GPU).

The fused model runs as chained custom autograd nodes (models/resnet.py ``_chain_blocks``) whose
parameter gradients arrive through the kernels' own backward; the DDP bucket hooks
(parallel/ddp.py) must still see every gradient, reduce it once and average it.  After
``finish()`` each rank's ``p.grad`` must equal the mean of the two ranks' single-process gradients
(bf16 tolerance) and be identical on both ranks.  RCCL refuses two ranks on one device, so the
ranks talk over gloo; the reduction path is the same code (reference DDP wrap:
harness/determined/pytorch/_pytorch_context.py:297)."""

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_ddp_over_fused_resnet50_averages_rank_gradients(tmp_path):
    port = _free_port()
    procs, outs = [], []
    for r in range(2):
        out = tmp_path / f"rank{r}.json"
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_ddp_fused_worker.py"), str(out)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
        outs.append(out)
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=240)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    reps = [json.loads(o.read_text()) for o in outs]
    for rep in reps:
        assert not rep["missing"], rep
        assert rep["n_params"] == 161, rep  # every ResNet-50 parameter got a reduced gradient
        assert rep["worst_rel_err"] < 3e-2, rep
        assert rep["same_as_rank0"], rep
    assert reps[0]["grad_norm"] == reps[1]["grad_norm"]
