#!/bin/bash
# GPT-2 ZeRO on one MI355X: GPU tests, benchmark sweep, kernel profile.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m pytest tests/test_zero_gpu.py -x -q > gpurun_out/zero_gpu_tests.log 2>&1 || { echo zero gpu tests failed; tail -40 gpurun_out/zero_gpu_tests.log; exit 1; }
tail -2 gpurun_out/zero_gpu_tests.log
for cfg in "--mb 8" "--mb 16" "--mb 8 --dropout 0"; do
  timeout -k 10 300 python -m determined_amd.benchmarks.gpt2 $cfg --steps 10 --warmup 3 > gpurun_out/gpt2_bench.log 2>&1 || { echo "gpt2 bench failed ($cfg)"; tail -30 gpurun_out/gpt2_bench.log; exit 1; }
  tail -1 gpurun_out/gpt2_bench.log
done
export TMPDIR=/tmp
rm -rf gpurun_out/prof_gpt2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt2 -o run --output-format csv -- python -m determined_amd.benchmarks.gpt2 --mb 8 --steps 5 --warmup 3 > gpurun_out/prof_gpt2.log 2>&1
echo "rocprof exit $?"
