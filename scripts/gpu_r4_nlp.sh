#!/bin/bash
# BASELINE configs #4/#5 on the current build: BERT-base MLM throughput fused vs stock + kernel profile,
# GPT-2 345M ZeRO-2 number + steady-state profile.
source "$(dirname "$0")/gpu_lib.sh"
step bert_bench 300 python -u scripts/bert_bench.py --batch 64 --seq 128 --steps 30 --warmup 10
rm -rf gpurun_out/prof_bert
step prof_bert 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run --output-format csv -- python scripts/bert_bench.py --variants fused --steps 8 --warmup 4
f=$(find gpurun_out/prof_bert -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python scripts/prof_steady.py "$f" --steps 6 --top 40 --marker adam_kernel > gpurun_out/prof_bert_summary.txt && head -30 gpurun_out/prof_bert_summary.txt
rm -f "$f"
step gpt2_bench 400 python -m determined_amd.benchmarks.gpt2 --mb 8 --steps 10 --warmup 3
step prof_gpt2 450 bash scripts/gpu_prof_gpt2.sh
exit $status
