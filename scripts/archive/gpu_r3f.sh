#!/bin/bash
# SQ counters of the 64-channel 56x56 3x3 halo forward (config 7, batch 1024), then the larger
# per-GPU batch sweep with MIOpen immediate mode.
set -o pipefail
cd "$(dirname "$0")/../.."
bash scripts/gpu_conv_pmc.sh "64 64 3 1 56 7 --batch 1024 --iters 10" "256 256 3 1 14 12 --batch 1024 --iters 10" > gpurun_out/r3f_pmc.txt 2>&1 || { tail -20 gpurun_out/r3f_pmc.txt; exit 1; }
cat gpurun_out/r3f_pmc.txt
bash scripts/archive/gpu_bs5.sh 1024 1536 2048
