#!/bin/bash
# GPU iteration: GPU tests (optional filter) -> bench variants -> rocprof kernel stats.
# usage: gpu_bench.sh "<pytest -k expr or empty>" "<variants>" "<bench extra args>" [profile_variant]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
K="$1"; VARIANTS="${2:-bf16_master}"; EXTRA="$3"; PROF="$4"
if [ -n "$K" ]; then
  timeout -k 10 500 python -m pytest tests -m gpu -x -q -k "$K" > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && { grep -E "Error|error|assert" gpurun_out/pytest_gpu.log | head -30; exit 1; }
fi
for v in $VARIANTS; do
  timeout -k 10 300 python bench.py --variant $v $EXTRA > gpurun_out/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -25 gpurun_out/bench_$v.log; exit 1; }
  tail -1 gpurun_out/bench_$v.log
done
if [ -n "$PROF" ]; then
  export TMPDIR=/tmp
  rm -rf gpurun_out/prof
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --variant $PROF $EXTRA --steps 10 --warmup 5 > gpurun_out/prof.log 2>&1
  echo "rocprof exit $?"
fi
