#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/ab_summary.txt
for ex in "" "wgrad:h0,wgrad:h1"; do
  DAMD_CONV_EXCLUDE="$ex" timeout -k 10 400 python bench.py --steps 30 --warmup 8 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  echo "exclude=[$ex] $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/ab_summary.txt
done
