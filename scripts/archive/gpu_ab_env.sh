#!/bin/bash
# Same-box interleaved A/B of the headline bench over one environment switch:
#   scripts/archive/gpu_ab_env.sh VAR VALUE_A VALUE_B [pytest -k expr]
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
var=$1; va=$2; vb=$3
if [ -n "$4" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "$4" --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
for v in "$va" "$vb" "$va" "$vb"; do
  env "$var=$v" timeout -k 10 330 python bench.py --steps 20 --warmup 5 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  echo "$var=$v $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/ab_summary.txt
done
