#!/bin/bash
# Fused-stem kernel counters + steady-state profile of the headline bench at batch 1024.
set -o pipefail
cd "$(dirname "$0")/../.."
bash scripts/archive/gpu_stem_prof.sh > gpurun_out/r3e_stem.txt 2>&1 || { tail -30 gpurun_out/r3e_stem.txt; exit 1; }
cat gpurun_out/r3e_stem.txt
bash scripts/gpu_prof_resnet.sh 1024
