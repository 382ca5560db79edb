#!/bin/bash
# Same-box A/B of the conv3x3v2 halo staging without a BN prologue: LDS-DMA (the default build) vs register
# staging (ab_reg/: HDMA off), forward with BN statistics and input gradient with the BN-backward epilogue.
source "$(dirname "$0")/gpu_lib.sh"
P="--passes fwd_stats,dgrad_bn_epi --batch 2048"
step hdma1 300 python -u scripts/v2_bench.py $P --out gpurun_out/hdma1.jsonl
export DAMD_AB_ROOT=$PWD/ab_reg
step reg1 300 python -u scripts/v2_bench.py $P --out gpurun_out/reg1.jsonl
unset DAMD_AB_ROOT
step hdma2 300 python -u scripts/v2_bench.py $P --out gpurun_out/hdma2.jsonl
export DAMD_AB_ROOT=$PWD/ab_reg
step reg2 300 python -u scripts/v2_bench.py $P --out gpurun_out/reg2.jsonl
exit $status
