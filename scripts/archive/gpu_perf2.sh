#!/bin/bash
# norm/bias-grad/attention tests, GPT-2 bench (plain and TunableOp), GPT-2 profile
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_attention_gpu.py tests/test_ops_gpu.py tests/test_zero_gpu.py -x -q > gpurun_out/perf2_tests.log 2>&1 || { echo tests failed; tail -60 gpurun_out/perf2_tests.log; exit 1; }
tail -2 gpurun_out/perf2_tests.log
timeout -k 10 300 python -m determined_amd.benchmarks.gpt2 --mb 8 --steps 10 --warmup 3 > gpurun_out/gpt2_b8.log 2>&1 || { echo gpt2 bench failed; tail -30 gpurun_out/gpt2_b8.log; exit 1; }
tail -1 gpurun_out/gpt2_b8.log
tail -1 gpurun_out/gpt2_b8_tun.log
export TMPDIR=/tmp
rm -rf gpurun_out/prof_gpt2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt2 -o run --output-format csv -- python -m determined_amd.benchmarks.gpt2 --mb 8 --steps 5 --warmup 3 > gpurun_out/prof_gpt2.log 2>&1
echo "rocprof exit $?"
