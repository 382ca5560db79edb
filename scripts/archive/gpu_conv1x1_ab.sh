#!/bin/bash
# conv1x1 GEMM input-gradient path: GPU numerics, then same-box bench A/B (on / off).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -x -q -k conv1x1 --timeout 120 --timeout-method thread > gpurun_out/c1_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/c1_tests.log; exit 1; }
tail -1 gpurun_out/c1_tests.log
: > gpurun_out/conv1x1_bench_ab.jsonl
for v in on off on off; do
  if [ $v = off ]; then export DAMD_DISABLE_FUSIONS=conv1x1_gemm; else unset DAMD_DISABLE_FUSIONS; fi
  timeout -k 10 300 python bench.py > gpurun_out/c1_bench.log 2>&1 || { echo "bench failed ($v)"; tail -20 gpurun_out/c1_bench.log; exit 1; }
  echo "{\"conv1x1_gemm\": \"$v\", \"bench\": $(grep '^{' gpurun_out/c1_bench.log)}" >> gpurun_out/conv1x1_bench_ab.jsonl
  tail -1 gpurun_out/c1_bench.log | cut -c1-200
done
