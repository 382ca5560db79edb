#!/bin/bash
# Round-4 baseline: launch-check GPU test, per-layer roofline at batch 2048, SQ counters of the 3x3 halo forwards.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_launch_check_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/launch_check.log 2>&1 || { tail -30 gpurun_out/launch_check.log; exit 1; }
tail -3 gpurun_out/launch_check.log
timeout -k 10 900 python -u scripts/layer_roofline.py --batch 2048 --out gpurun_out/roofline_b2048.jsonl > gpurun_out/roofline_b2048.log 2>&1 || { tail -20 gpurun_out/roofline_b2048.log; exit 1; }
tail -1 gpurun_out/roofline_b2048.jsonl
bash scripts/gpu_conv_pmc.sh "64 64 3 1 56 19 --batch 2048 --iters 10" "128 128 3 1 28 18 --batch 2048 --iters 10" "256 256 3 1 14 18 --batch 2048 --iters 10" > gpurun_out/pmc_halo_b2048.txt 2>&1
cat gpurun_out/pmc_halo_b2048.txt
