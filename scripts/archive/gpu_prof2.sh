#!/bin/bash
# Warm MIOpen's find-db with one bench run, save the db, then profile steady state.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
mkdir -p $MIOPEN_USER_DB_PATH
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_warm.log 2>&1 || { tail -20 gpurun_out/bench_warm.log; exit 1; }
tail -1 gpurun_out/bench_warm.log
ls -la $MIOPEN_USER_DB_PATH
timeout -k 10 400 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_cached.log 2>&1 || { tail -20 gpurun_out/bench_cached.log; exit 1; }
tail -1 gpurun_out/bench_cached.log
export TMPDIR=/tmp
rm -rf gpurun_out/prof_s
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s -o run --output-format csv -- python bench.py --steps 10 --warmup 3 > gpurun_out/prof_s.log 2>&1
echo "rocprof exit $?"
