#!/bin/bash
# GPU iteration: selected GPU tests (pytest -k expr) then the 1-GPU headline bench.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
K="$1"
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_q.log 2>&1
  rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_q.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_q.log | head -30; exit 1; }
fi
timeout -k 10 500 python bench.py --steps 20 --warmup 8 ${@:2} > gpurun_out/bench_q.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench_q.log; exit 1; }
tail -1 gpurun_out/bench_q.log
