#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > gpurun_out/phase_tests.log 2>&1 || { echo "conv tests failed"; tail -30 gpurun_out/phase_tests.log; exit 1; }
tail -1 gpurun_out/phase_tests.log
timeout -k 10 300 python scripts/archive/dgrad_s2_time.py 1024 2>&1 | grep -v amdgpu.ids
