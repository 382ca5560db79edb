#!/bin/bash
# conv3x3v2: RES halo transformed in halves during the taps (only LDS stores at the unit boundary): correctness, per-config timing, bench.
# correctness, per-config timing, SQ counters of the resident config, headline bench.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step v10_tests 300 $PYT --timeout 120 tests/test_conv3x3v2_gpu.py
[ $status -ne 0 ] && exit 1
step v10_bench 420 python -u scripts/v2_bench.py --batch 2048 --out gpurun_out/v10_bench.jsonl
step bench 360 python bench.py --steps 20 --warmup 5
exit $status
