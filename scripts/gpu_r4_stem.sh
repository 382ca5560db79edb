#!/bin/bash
# Stem pooling on sign-flipped keys: stem / BN / training-curve tests, stem kernel timing, headline bench.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step stem_tests 400 $PYT --timeout 200 tests/test_bn_gpu.py tests/test_ops_gpu.py tests/test_resnet_training_gpu.py -k "stem or pool or training"
[ $status -ne 0 ] && exit 1
step stem_time 200 python -u scripts/stem_time.py --batch 2048
step bench 300 python bench.py --steps 20 --warmup 5
exit $status
