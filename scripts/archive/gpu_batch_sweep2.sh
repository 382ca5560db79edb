#!/bin/bash
# ResNet-50 per-GPU batch sweep on one MI355X (288 GB HBM lets the batch grow well past 512).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for B in "$@"; do
  timeout -k 10 420 python bench.py --steps 15 --warmup 6 --batch $B > gpurun_out/bench_b$B.log 2>&1 || { echo "batch $B failed"; tail -5 gpurun_out/bench_b$B.log; exit 1; }
  tail -1 gpurun_out/bench_b$B.log
done
