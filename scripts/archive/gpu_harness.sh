#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_harness.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench_harness.log; exit 1; }
tail -1 gpurun_out/bench_harness.log
timeout -k 10 400 python bench.py --steps 30 --warmup 10 --no-harness > gpurun_out/bench_direct.log 2>&1 || { echo bench2 failed; tail -30 gpurun_out/bench_direct.log; exit 1; }
tail -1 gpurun_out/bench_direct.log
export TMPDIR=/tmp
rm -rf gpurun_out/prof_h
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_h -o run --output-format csv -- python bench.py --steps 10 --warmup 10 > gpurun_out/prof_h.log 2>&1
echo "rocprof exit $?"
