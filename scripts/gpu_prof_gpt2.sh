#!/bin/bash
# GPT-2 345M ZeRO-2 mb8 steady-state kernel profile + last-step launch sequence with gaps.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
rm -rf gpurun_out/prof_g
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g -o run --output-format csv -- python -m determined_amd.benchmarks.gpt2 --mb 8 --steps 6 --warmup 3 > gpurun_out/prof_g.log 2>&1 || { echo gpt2 profile failed; tail -5 gpurun_out/prof_g.log; exit 1; }
f=$(find gpurun_out/prof_g -name "*kernel_trace.csv" | head -1)
python scripts/prof_steady.py "$f" --steps 3 --top 40 --marker adam_kernel --seq gpurun_out/prof_g_seq.txt > gpurun_out/prof_g_summary.txt && head -3 gpurun_out/prof_g_summary.txt
rm -f "$f"
