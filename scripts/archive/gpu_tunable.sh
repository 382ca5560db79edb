#!/bin/bash
# Same-box A/B of GPT-2 345M with hipBLASLt's default GEMM choice vs the in-tree TunableOp
# results (determined_amd/benchmarks/tunableop/, searched with --tune).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
f=determined_amd/benchmarks/tunableop/gpt2_345m_mb8.csv
for mode in base tuned base tuned; do
  extra=""; [ $mode = tuned ] && extra="--tunable $f"
  timeout -k 10 200 python -m determined_amd.benchmarks.gpt2 --mb 8 --steps 10 --warmup 3 $extra > gpurun_out/tun_$mode.log 2>&1 || { tail -5 gpurun_out/tun_$mode.log; exit 1; }
  echo "$mode $(tail -1 gpurun_out/tun_$mode.log | cut -c1-120)"
done
