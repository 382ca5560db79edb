#!/bin/bash
# conv3x3v2 8-wave: single-shot halo stored at tap 5, PRO coefficients in LDS: correctness, per-config timing, bench.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step v6_tests 300 $PYT --timeout 120 tests/test_conv3x3v2_gpu.py
[ $status -ne 0 ] && exit 1
step v6_bench 420 python -u scripts/v2_bench.py --batch 2048 --out gpurun_out/v6_bench.jsonl
step bench 360 python bench.py --steps 20 --warmup 5
exit $status
