#!/bin/bash
# GPU tests matching $1 (pytest -k), then a same-box interleaved A/B of the headline bench with the
# conv candidates in $2 (DAMD_CONV_EXCLUDE syntax) excluded vs allowed: excluded, allowed, x2.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -n "$1" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "$1" --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
for ex in "$2" "" "$2" ""; do
  DAMD_CONV_EXCLUDE="$ex" timeout -k 10 400 python bench.py --steps 30 --warmup 8 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  echo "exclude=[$ex] $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/ab_summary.txt
done
