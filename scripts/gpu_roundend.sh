#!/bin/bash
# Rehearsal of the driver's round-end GPU tiers: full GPU test suite, smoke(), default bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/re_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/re_pytest.log; exit 1; }
tail -1 gpurun_out/re_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/re_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/re_smoke.log; exit 1; }
tail -1 gpurun_out/re_smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/re_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/re_bench.log; exit 1; }
tail -1 gpurun_out/re_bench.log
