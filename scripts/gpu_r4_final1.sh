#!/bin/bash
# Round-4 end-of-work evidence: per-layer roofline table at batch 2048 with the round-4 kernels, and the BERT
# bf16-weights step profile.
source "$(dirname "$0")/gpu_lib.sh"
step roofline 900 python -u scripts/layer_roofline.py --batch 2048 --out gpurun_out/roofline_b2048_r4_end.jsonl
tail -1 gpurun_out/roofline_b2048_r4_end.jsonl
rm -rf gpurun_out/prof_bert2
step prof_bert2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert2 -o run --output-format csv -- python scripts/bert_bench.py --variants fused_bf16w --steps 8 --warmup 4
f=$(find gpurun_out/prof_bert2 -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && python scripts/prof_steady.py "$f" --steps 6 --top 30 --marker adam_kernel > gpurun_out/prof_bert2_summary.txt && head -8 gpurun_out/prof_bert2_summary.txt
rm -f "$f"
exit $status
