#!/bin/bash
# Compute-stream priority vs simulated collective interference (scripts/dev/bench_interference.py).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in "|" "1|" "|16:200" "1|16:200"; do
  hp=${cfg%%|*}; sim=${cfg#*|}
  DAMD_SIM_HIPRIO=$hp DAMD_SIM_COLLECTIVE="$sim" timeout -k 10 400 python scripts/dev/bench_interference.py --steps 30 --warmup 8 > gpurun_out/pr.log 2>&1 || { tail -20 gpurun_out/pr.log; exit 1; }
  echo "hiprio=[$hp] sim=[$sim] $(tail -1 gpurun_out/pr.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/pr_summary.txt
done
