#!/bin/bash
# BN apply passes with two vectors in flight per thread: BN tests, same-box apply bandwidth old build
# (ab_old/, the previous kernels) vs new, then the headline bench on the new build.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step bn_tests 300 $PYT --timeout 120 tests/test_bn_gpu.py
[ $status -ne 0 ] && exit 1
export DAMD_AB_ROOT=$PWD/ab_old
step bnbw_old1 200 python -u scripts/bn_apply_bw.py
unset DAMD_AB_ROOT
step bnbw_new1 200 python -u scripts/bn_apply_bw.py
export DAMD_AB_ROOT=$PWD/ab_old
step bnbw_old2 200 python -u scripts/bn_apply_bw.py
unset DAMD_AB_ROOT
step bnbw_new2 200 python -u scripts/bn_apply_bw.py
step bench 300 python bench.py --steps 20 --warmup 5
exit $status
