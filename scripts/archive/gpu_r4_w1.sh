#!/bin/bash
# conv3x3v2 whole-row-tile weight gradient: correctness of every v2 test, per-config wgrad timing at the bench batch.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step w1_tests 300 $PYT --timeout 120 tests/test_conv3x3v2_gpu.py tests/test_conv_gpu.py -k "wgrad"
[ $status -ne 0 ] && exit 1
step w1_bench 420 python -u scripts/v2_bench.py --batch 2048 --passes wgrad --out gpurun_out/w1_bench.jsonl
exit $status
