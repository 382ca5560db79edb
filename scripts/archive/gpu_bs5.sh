#!/bin/bash
# Per-GPU batch sweep with MIOpen's immediate-mode solver choice (no find-db search: the in-tree
# find-db only holds the batch-1024 shapes), so larger batches start within minutes.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for b in ${@:-1024 1536 2048}; do
  timeout -k 10 700 python bench.py --batch $b --steps 10 --warmup 3 --conv-benchmark 0 > gpurun_out/bs5_$b.log 2>&1 || { echo "batch $b failed"; grep -v "warming up" gpurun_out/bs5_$b.log | tail -20; exit 1; }
  echo "batch $b: $(grep peak gpurun_out/bs5_$b.log) $(tail -1 gpurun_out/bs5_$b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/bs5_summary.txt
done
