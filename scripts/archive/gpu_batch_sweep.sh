#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for b in 384 512 768; do
  timeout -k 10 500 python bench.py --steps 20 --warmup 8 --batch $b > gpurun_out/bench_b$b.log 2>&1 || { echo "bench $b failed"; tail -20 gpurun_out/bench_b$b.log; exit 1; }
  tail -1 gpurun_out/bench_b$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($b, d['value'], d['ms_per_step'])"
done
