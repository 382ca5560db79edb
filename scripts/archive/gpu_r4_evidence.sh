#!/bin/bash
# Headline bench + steady-state ResNet-50 profile at the bench batch, then BERT-base (config #5)
# throughput fused vs stock and its kernel profile.
source "$(dirname "$0")/gpu_lib.sh"
step bench 420 python bench.py --steps 20 --warmup 5
step bench256 300 python bench.py --batch 256 --steps 30 --warmup 8
step prof_resnet 600 bash scripts/gpu_prof_resnet.sh 2048
step bert_bench 300 python -u scripts/bert_bench.py --batch 64 --seq 128 --steps 30 --warmup 10
rm -rf gpurun_out/prof_bert
step prof_bert 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run --output-format csv -- python scripts/bert_bench.py --variants fused --steps 8 --warmup 4
f=$(find gpurun_out/prof_bert -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python scripts/prof_steady.py "$f" --steps 6 --top 40 --marker adam_kernel > gpurun_out/prof_bert_summary.txt && head -30 gpurun_out/prof_bert_summary.txt
rm -f "$f"
exit $status
