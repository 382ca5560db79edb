#!/bin/bash
# Larger per-GPU batches of the headline bench (288 GB HBM3E: batch 1024 uses ~120 GB).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for b in ${@:-1536 2048}; do
  timeout -k 10 540 python bench.py --batch $b --steps 10 --warmup 4 > gpurun_out/bs_$b.log 2>&1 || { echo "batch $b failed"; tail -20 gpurun_out/bs_$b.log; exit 1; }
  tail -1 gpurun_out/bs_$b.log | tee -a gpurun_out/bs4_summary.jsonl
  python -c "import torch; print('peak mem GB', torch.cuda.mem_get_info())" > /dev/null 2>&1
done
