#!/bin/bash
# Weight-gradient configs: GPU numerics, per-layer timings vs MIOpen (ResNet-50 shapes, b512), bench.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 200 --timeout-method thread -k wgrad > gpurun_out/wg_tests.log 2>&1 || { tail -30 gpurun_out/wg_tests.log; exit 1; }
tail -1 gpurun_out/wg_tests.log
rm -f gpurun_out/conv_wgrad.jsonl
timeout -k 10 500 python scripts/conv_bench.py --only wgrad --out gpurun_out/conv_wgrad.jsonl > gpurun_out/conv_wgrad.log 2>&1 || { tail -20 gpurun_out/conv_wgrad.log; exit 1; }
tail -1 gpurun_out/conv_wgrad.log
timeout -k 10 600 python bench.py > gpurun_out/wg_bench.log 2>&1 || { tail -20 gpurun_out/wg_bench.log; exit 1; }
tail -1 gpurun_out/wg_bench.log
