#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python scripts/conv_sweep.py 256 0 > gpurun_out/conv_sweep_default.log 2>&1 || { tail -20 gpurun_out/conv_sweep_default.log; exit 1; }
tail -1 gpurun_out/conv_sweep_default.log
timeout -k 10 500 python scripts/conv_sweep.py 256 1 > gpurun_out/conv_sweep_bench.log 2>&1 || { tail -20 gpurun_out/conv_sweep_bench.log; exit 1; }
tail -1 gpurun_out/conv_sweep_bench.log
timeout -k 10 400 python bench.py --no-harness --variant bf16_master --steps 20 --warmup 8 --conv-benchmark 1 > gpurun_out/bench_convbench.log 2>&1 || { tail -20 gpurun_out/bench_convbench.log; exit 1; }
tail -1 gpurun_out/bench_convbench.log
