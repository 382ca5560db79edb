#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m pytest tests/test_attention_gpu.py -x -q > gpurun_out/attn_tests.log 2>&1 || { echo attn tests failed; tail -60 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
timeout -k 10 300 python scripts/attn_bench.py > gpurun_out/attn_bench.log 2>&1 || { echo attn bench failed; tail -30 gpurun_out/attn_bench.log; exit 1; }
cat gpurun_out/attn_bench.log | grep shape
timeout -k 10 300 python -m determined_amd.benchmarks.gpt2 --mb 8 --steps 10 --warmup 3 > gpurun_out/gpt2_bench.log 2>&1 || { echo gpt2 bench failed; tail -30 gpurun_out/gpt2_bench.log; exit 1; }
tail -1 gpurun_out/gpt2_bench.log
timeout -k 10 300 python -m determined_amd.benchmarks.gpt2 --mb 16 --steps 10 --warmup 3 > gpurun_out/gpt2_bench16.log 2>&1 || { echo gpt2 bench16 failed; tail -30 gpurun_out/gpt2_bench16.log; exit 1; }
tail -1 gpurun_out/gpt2_bench16.log
export TMPDIR=/tmp
rm -rf gpurun_out/prof_gpt2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt2 -o run --output-format csv -- python -m determined_amd.benchmarks.gpt2 --mb 8 --steps 5 --warmup 3 > gpurun_out/prof_gpt2.log 2>&1
echo "rocprof exit $?"
