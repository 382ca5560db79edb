#!/bin/bash
# Persistent-grid oversubscription vs collective interference (1 GPU): bench with and without a
# simulated bucket collective (scripts/dev/bench_interference.py) for DAMD_CONV_OVERSUB=1 / k.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
K=${1:-3}
for cfg in "1|" "$K|" "1|16:200" "$K|16:200"; do
  ov=${cfg%%|*}; sim=${cfg#*|}
  DAMD_CONV_OVERSUB=$ov DAMD_SIM_COLLECTIVE="$sim" timeout -k 10 400 python scripts/dev/bench_interference.py --steps 30 --warmup 8 > gpurun_out/ov.log 2>&1 || { tail -20 gpurun_out/ov.log; exit 1; }
  echo "oversub=$ov sim=[$sim] $(tail -1 gpurun_out/ov.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/ov_summary.txt
done
