#!/bin/bash
# Steady-state rocprofv3 kernel summaries of the two benchmark models (-> gpurun_out/*_summary.txt).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
bash scripts/gpu_prof_resnet.sh 512 > /dev/null || { echo resnet profile failed; exit 1; }
head -3 gpurun_out/prof_r_summary.txt
rm -rf gpurun_out/prof_g
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g -o run --output-format csv -- python -m determined_amd.benchmarks.gpt2 --mb 8 --steps 6 --warmup 3 > gpurun_out/prof_g.log 2>&1 || { echo gpt2 profile failed; tail -5 gpurun_out/prof_g.log; exit 1; }
f=$(find gpurun_out/prof_g -name "*kernel_trace.csv" | head -1)
python scripts/prof_steady.py "$f" --steps 3 --top 40 --marker adam_kernel --seq gpurun_out/prof_g_seq.txt > gpurun_out/prof_g_summary.txt && head -3 gpurun_out/prof_g_summary.txt
rm -f "$f"
