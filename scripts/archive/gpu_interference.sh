#!/bin/bash
# Collective/compute interference rehearsal on one GPU (scripts/dev/bench_interference.py).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for sim in "" "16:200" "32:200" "16:200:end" ""; do
  DAMD_SIM_COLLECTIVE="$sim" timeout -k 10 400 python scripts/dev/bench_interference.py --steps 30 --warmup 8 > gpurun_out/if.log 2>&1 || { tail -20 gpurun_out/if.log; exit 1; }
  echo "sim=[$sim] $(tail -1 gpurun_out/if.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/if_summary.txt
done
