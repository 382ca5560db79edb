#!/bin/bash
# conv3x3v2 weight gradient incl. the 7x7 configs (h8 DMA / h9 register-staged): tests, per-config timing
# of the 7x7 layer (512 channels) and the 56x56 layer, then the headline bench.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step w4_tests 300 $PYT --timeout 120 tests/test_conv3x3v2_gpu.py tests/test_conv_gpu.py -k "wgrad"
[ $status -ne 0 ] && exit 1
step w4_bench 420 python -u scripts/v2_bench.py --batch 2048 --passes wgrad --layers 512x7,64x56 --out gpurun_out/w4_bench.jsonl
step bench 300 python bench.py --steps 20 --warmup 5
exit $status
