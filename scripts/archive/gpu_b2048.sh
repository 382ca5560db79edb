#!/bin/bash
# Batch 2048 with the in-tree find-db: MIOpen find (benchmark=1) vs immediate mode, same box.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cb in 1 0 1 0; do
  timeout -k 10 560 python bench.py --batch 2048 --steps 15 --warmup 4 --conv-benchmark $cb > gpurun_out/b2048_$cb.log 2>&1 || { echo "cb=$cb failed"; grep -v "warming up" gpurun_out/b2048_$cb.log | tail -5; exit 1; }
  echo "conv-benchmark=$cb $(grep tuned gpurun_out/b2048_$cb.log) $(tail -1 gpurun_out/b2048_$cb.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/b2048_summary.txt
done
