#!/bin/bash
# conv3x3v2 with both wave counts (4 waves at 1/SIMD, 8 waves at 2/SIMD, same chunk-planar layout):
# correctness of every config, per-config timing at the bench batch, then the headline bench.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step v4_tests 300 $PYT --timeout 120 tests/test_conv3x3v2_gpu.py
[ $status -ne 0 ] && exit 1
step v4_bench 420 python -u scripts/v2_bench.py --batch 2048 --out gpurun_out/v4_bench.jsonl
step bench 360 python bench.py --steps 20 --warmup 5
exit $status
