#!/bin/bash
# conv3x3v2 weight gradient: DMA (h2-h4) vs register-staged line-coalesced loads (h5-h7): tests, per-config timing.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step w3_tests 300 $PYT --timeout 120 tests/test_conv3x3v2_gpu.py tests/test_conv_gpu.py -k "wgrad"
[ $status -ne 0 ] && exit 1
step w3_bench 420 python -u scripts/v2_bench.py --batch 2048 --passes wgrad --out gpurun_out/w3_bench.jsonl
exit $status
