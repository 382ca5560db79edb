#!/bin/bash
# Rehearsal of bench.py's multi-rank path on a 1-GPU box: 2 torchrun ranks share the GPU and
# talk over gloo (RCCL refuses two ranks on one device).  Checks the JSON contract for N=2.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
DAMD_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --batch 64 \
  > gpurun_out/mr.out 2> gpurun_out/mr.err || { tail -30 gpurun_out/mr.err; exit 1; }
cat gpurun_out/mr.out
python - <<'PY'
import json
lines = [l for l in open("gpurun_out/mr.out") if l.strip()]
assert len(lines) == 1, lines
d = json.loads(lines[0])
assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 128 and d["config"]["parallelism"] == "dp2", d
print("multi-rank contract ok")
PY
