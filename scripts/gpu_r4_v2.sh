#!/bin/bash
# conv3x3v2: correctness vs fp32, then per-config timing at the bench batch and SQ counters of the v2 forward.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv3x3v2_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/v2_tests.log 2>&1 || { tail -40 gpurun_out/v2_tests.log; exit 1; }
tail -3 gpurun_out/v2_tests.log
timeout -k 10 600 python -u scripts/v2_bench.py --batch 2048 --out gpurun_out/v2_bench.jsonl > gpurun_out/v2_bench.log 2>&1 || { tail -20 gpurun_out/v2_bench.log; exit 1; }
cat gpurun_out/v2_bench.jsonl
