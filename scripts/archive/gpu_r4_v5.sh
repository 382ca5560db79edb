#!/bin/bash
# conv3x3v2 8-wave configs with single-buffered fragments (no spills at 2 waves/SIMD): correctness, per-config timing.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step v5_tests 300 $PYT --timeout 120 tests/test_conv3x3v2_gpu.py
[ $status -ne 0 ] && exit 1
step v5_bench 420 python -u scripts/v2_bench.py --batch 2048 --out gpurun_out/v5_bench.jsonl
exit $status
