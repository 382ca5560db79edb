#!/bin/bash
# Harvest the MIOpen find-db for the ResNet-50 bench (batch 512) and check the warm-up speedup.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/miopen_db
export HSA_ENABLE_IPC_MODE_LEGACY=0
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
timeout -k 10 900 python bench.py --steps 20 --warmup 8 > gpurun_out/bench_b512_a.log 2> gpurun_out/bench_b512_a.err || { echo bench a failed; tail -20 gpurun_out/bench_b512_a.err; exit 1; }
tail -1 gpurun_out/bench_b512_a.log; grep warmup gpurun_out/bench_b512_a.err | tail -2
timeout -k 10 900 python bench.py --steps 20 --warmup 8 > gpurun_out/bench_b512_b.log 2> gpurun_out/bench_b512_b.err || { echo bench b failed; tail -20 gpurun_out/bench_b512_b.err; exit 1; }
tail -1 gpurun_out/bench_b512_b.log; grep warmup gpurun_out/bench_b512_b.err | tail -2
ls -la gpurun_out/miopen_db
