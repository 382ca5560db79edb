#!/bin/bash
# First MI355X pass: kernel numerics, bench variants, rocprof kernel stats.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?" | tee -a gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
for v in bf16_master bf16_fp32bn amp; do
  timeout -k 10 300 python bench.py --no-harness --variant $v --steps 20 --warmup 8 > gpurun_out/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/bench_$v.log; exit 1; }
  tail -1 gpurun_out/bench_$v.log
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet -o run --output-format csv -- python bench.py --no-harness --variant bf16_master --steps 10 --warmup 5 > gpurun_out/prof.log 2>&1
echo "rocprof exit $?"
find gpurun_out/prof_resnet -name "*stats*" | head
