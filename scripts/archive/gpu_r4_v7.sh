#!/bin/bash
# conv3x3v2 8-wave: halo via buffer loads (per-unit resource, out-of-range offsets give the zero padding): correctness, per-config timing, bench.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step v7_tests 300 $PYT --timeout 120 tests/test_conv3x3v2_gpu.py
[ $status -ne 0 ] && exit 1
step v7_bench 420 python -u scripts/v2_bench.py --batch 2048 --out gpurun_out/v7_bench.jsonl
step bench 360 python bench.py --steps 20 --warmup 5
exit $status
