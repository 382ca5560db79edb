#!/bin/bash
# Round 3: the new GPU tests first, then rehearsal + per-layer roofline.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_resnet_training_gpu.py tests/test_ops_gpu.py -k "hooked or unscale or follows" > gpurun_out/new_tests.log 2>&1 || { echo "new tests failed"; tail -30 gpurun_out/new_tests.log; exit 1; }
tail -2 gpurun_out/new_tests.log
bash scripts/archive/gpu_r3a.sh
