#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/pretune_ab.txt
for mode in pretune instep pretune instep; do
  extra=""; [ "$mode" = instep ] && extra="--no-pretune"
  timeout -k 10 400 python bench.py --steps 30 --warmup 6 $extra > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
  echo "$mode $(tail -1 gpurun_out/pt.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/pretune_ab.txt
done
