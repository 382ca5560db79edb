#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 200 --timeout-method thread -k "halo_wgrad" > gpurun_out/wg3_tests.log 2>&1 || { tail -40 gpurun_out/wg3_tests.log; exit 1; }
tail -1 gpurun_out/wg3_tests.log
rm -f gpurun_out/conv_wgrad3.jsonl
timeout -k 10 400 python scripts/conv_bench.py --only wgrad --shapes 1,5,9,11,15,17,21 --out gpurun_out/conv_wgrad3.jsonl > gpurun_out/conv_wgrad3.log 2>&1 || { tail -20 gpurun_out/conv_wgrad3.log; exit 1; }
tail -1 gpurun_out/conv_wgrad3.log
