#!/bin/bash
# Stem kernel timing at the bench batch (fused conv+BN+ReLU+max-pool vs the unfused kernels).
source "$(dirname "$0")/gpu_lib.sh"
step stem_time 200 python -u scripts/stem_time.py --batch 2048
exit $status
