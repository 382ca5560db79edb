#!/bin/bash
# Per-GPU batch sweep of the headline bench with the current kernels (one box).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for b in 256 512 1024; do
  timeout -k 10 500 python bench.py --batch $b --steps 20 --warmup 5 > gpurun_out/bs.log 2>&1 || { tail -20 gpurun_out/bs.log; exit 1; }
  tail -1 gpurun_out/bs.log | tee -a gpurun_out/bs_summary.jsonl
done
