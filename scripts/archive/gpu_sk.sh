#!/bin/bash
# Stream-K A/B: per-layer forward / input-gradient timings of every config (ResNet-50 shapes, b512),
# then the headline bench with the tuner free to pick stream-K configs.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/conv_sk.jsonl
timeout -k 10 500 python scripts/conv_bench.py --only fwd --out gpurun_out/conv_sk.jsonl > gpurun_out/conv_sk_fwd.log 2>&1 || { tail -20 gpurun_out/conv_sk_fwd.log; exit 1; }
tail -1 gpurun_out/conv_sk_fwd.log
timeout -k 10 500 python scripts/conv_bench.py --only dgrad --out gpurun_out/conv_sk.jsonl > gpurun_out/conv_sk_dgrad.log 2>&1 || { tail -20 gpurun_out/conv_sk_dgrad.log; exit 1; }
tail -1 gpurun_out/conv_sk_dgrad.log
timeout -k 10 600 python bench.py > gpurun_out/sk_bench.log 2>&1 || { tail -20 gpurun_out/sk_bench.log; exit 1; }
tail -1 gpurun_out/sk_bench.log
