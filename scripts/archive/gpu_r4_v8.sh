#!/bin/bash
# conv3x3v2: buffer-load halo staging, LDS-DMA halo for PRO=0, 64x64-wave-tile configs (56x56 8-row single halo, 28x28 7-row): correctness, per-config timing, bench.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step v8_tests 300 $PYT --timeout 120 tests/test_conv3x3v2_gpu.py
[ $status -ne 0 ] && exit 1
step v8_bench 420 python -u scripts/v2_bench.py --batch 2048 --out gpurun_out/v8_bench.jsonl
step bench 360 python bench.py --steps 20 --warmup 5
exit $status
