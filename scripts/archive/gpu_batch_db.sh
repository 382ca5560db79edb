#!/bin/bash
# Per-GPU batch B on one MI355X: MIOpen solver search into a scratch find-db (seeded with the
# in-tree one), then a second run that reuses it.  The db lands in gpurun_out/miopen_db.
set -o pipefail
cd "$(dirname "$0")/../.."
B=${1:-1024}
mkdir -p gpurun_out/miopen_db
cp -n determined_amd/benchmarks/miopen_db/* gpurun_out/miopen_db/ 2>/dev/null
export HSA_ENABLE_IPC_MODE_LEGACY=0
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
timeout -k 10 900 python bench.py --steps 10 --warmup 4 --batch $B > gpurun_out/bench_b${B}_search.log 2>&1 || { echo search failed; tail -5 gpurun_out/bench_b${B}_search.log; exit 1; }
tail -1 gpurun_out/bench_b${B}_search.log
timeout -k 10 600 python bench.py --steps 20 --warmup 6 --batch $B > gpurun_out/bench_b${B}.log 2>&1 || { echo bench failed; tail -5 gpurun_out/bench_b${B}.log; exit 1; }
tail -1 gpurun_out/bench_b${B}.log
grep "warmup 1/" gpurun_out/bench_b${B}.log
