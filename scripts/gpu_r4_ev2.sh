#!/bin/bash
# Round-4 evidence after the conv3x3v2 work: same-box A/B, batch-256 number, steady-state ResNet-50 profile.
source "$(dirname "$0")/gpu_lib.sh"
step ab 1000 bash scripts/gpu_r4_ab.sh
unset DAMD_CONV_EXCLUDE
step bench256 300 python bench.py --batch 256 --steps 30 --warmup 8
step prof_resnet 600 bash scripts/gpu_prof_resnet.sh 2048
exit $status
