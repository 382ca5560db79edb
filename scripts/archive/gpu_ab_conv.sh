#!/bin/bash
# Same-box A/B of new conv configs: the headline bench with each family excluded from the tuner.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for ex in "" "wgrad:8-11" "*:14-21" "wgrad:8-11,*:14-21"; do
  DAMD_CONV_EXCLUDE="$ex" timeout -k 10 400 python bench.py --steps 30 --warmup 8 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  echo "exclude=[$ex] $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/ab_summary.txt
done
