#!/bin/bash
# Restructured conv3x3v2 (4 waves, 64x64 wave tiles, chunk-planar halo, 5-slot weight ring): correctness,
# per-config timing, SQ counters of the 56x56 forward, then the headline bench.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step v3_tests 240 $PYT --timeout 120 tests/test_conv3x3v2_gpu.py
[ $status -ne 0 ] && exit 1
step v3_bench 300 python -u scripts/v2_bench.py --batch 2048 --out gpurun_out/v3_bench.jsonl
step pmc_v3 200 bash scripts/gpu_conv_pmc.sh "64 64 3 1 56 26 --batch 2048 --iters 10" "128 128 3 1 28 27 --batch 2048 --iters 10"
step bench 300 python bench.py --steps 20 --warmup 5
exit $status
