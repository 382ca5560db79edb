#!/bin/bash
# conv3x3v2: resident 64-channel filter (no per-tap barrier) for the 56x56 layer, packed-fp32 BN statistics:
# correctness, per-config timing, SQ counters of the resident config, headline bench.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step v9_tests 300 $PYT --timeout 120 tests/test_conv3x3v2_gpu.py
[ $status -ne 0 ] && exit 1
step v9_bench 420 python -u scripts/v2_bench.py --batch 2048 --out gpurun_out/v9_bench.jsonl
step pmc_v9 200 bash scripts/gpu_conv_pmc.sh "64 64 3 1 56 32 --batch 2048 --iters 10"
step bench 360 python bench.py --steps 20 --warmup 5
exit $status
