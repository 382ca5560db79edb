#!/bin/bash
# Current-tree GPT-2 345M ZeRO-2 throughput check on one MI355X (mb 8 and 16).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
: > gpurun_out/gpt2_check.jsonl
for mb in 8 16; do
  timeout -k 10 300 python -m determined_amd.benchmarks.gpt2 --mb $mb --steps 10 --warmup 3 > gpurun_out/gpt2_check_$mb.log 2>&1 || { echo "gpt2 bench failed (mb $mb)"; tail -30 gpurun_out/gpt2_check_$mb.log; exit 1; }
  grep '^{' gpurun_out/gpt2_check_$mb.log >> gpurun_out/gpt2_check.jsonl
  tail -1 gpurun_out/gpt2_check_$mb.log
done
