#!/bin/bash
# SQ counters of the 3x3 stride-1 forward at batch 2048 (64x64 @ 56x56): conv3x3v2 (cfg 26) vs the
# conv_igemm.hip halo / generic kernels the tuner used before (cfg 7, 6), then the per-layer roofline.
source "$(dirname "$0")/gpu_lib.sh"
step pmc 400 bash scripts/gpu_conv_pmc.sh "64 64 3 1 56 26 --batch 2048 --iters 10" "64 64 3 1 56 7 --batch 2048 --iters 10" "128 128 3 1 28 27 --batch 2048 --iters 10" "128 128 3 1 28 6 --batch 2048 --iters 10"
step roofline 600 python -u scripts/layer_roofline.py --batch 2048 --out gpurun_out/roofline_b2048_r4.jsonl
tail -1 gpurun_out/roofline_b2048_r4.jsonl
exit $status
