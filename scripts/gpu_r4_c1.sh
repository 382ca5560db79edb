#!/bin/bash
# conv3x3v2 tests incl. the NB=1 / 7-row shapes, SQ counters of the 64x64-tile configs, then the 2-rank
# batch-2048 rehearsal (JSON contract, gloo-agreed tuning time).
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step c1_tests 300 $PYT --timeout 120 tests/test_conv3x3v2_gpu.py
[ $status -ne 0 ] && exit 1
step pmc_v8 300 bash scripts/gpu_conv_pmc.sh "64 64 3 1 56 30 --batch 2048 --iters 10" "64 64 3 1 56 26 --batch 2048 --iters 10" "256 256 3 1 14 29 --batch 2048 --iters 10"
step multirank 600 bash scripts/gpu_multirank_b2048.sh
grep -E "tuned|timing candidates|warmup 1/" gpurun_out/mr2k.err | head -6
exit $status
