#!/bin/bash
# One GPU iteration: kernel tests touched by the change -> ResNet-50 bench -> GPT-2 bench.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_attention_gpu.py tests/test_bn_gpu.py tests/test_ops_gpu.py tests/test_zero_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/pytest_iter.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_iter.log | head -30; exit 1; }
timeout -k 10 500 python bench.py --steps 20 --warmup 8 > gpurun_out/bench_iter.log 2>&1 || { echo bench failed; tail -20 gpurun_out/bench_iter.log; exit 1; }
tail -1 gpurun_out/bench_iter.log
for cfg in "--mb 8" "--mb 16"; do
  timeout -k 10 300 python -m determined_amd.benchmarks.gpt2 $cfg --steps 10 --warmup 3 > gpurun_out/gpt2_iter.log 2>&1 || { echo "gpt2 bench failed ($cfg)"; tail -20 gpurun_out/gpt2_iter.log; exit 1; }
  tail -1 gpurun_out/gpt2_iter.log
done
