#!/bin/bash
# Software-pipelined generic conv configs (22-25) vs their SCH-0 twins (1, 5, 3, 4): numerics,
# per-layer timings, then a same-box bench A/B with the new configs excluded / allowed.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gpu.py tests/test_bn_gpu.py > gpurun_out/sch3_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/sch3_tests.log; exit 1; }
tail -1 gpurun_out/sch3_tests.log
for spec in "64 256 1 1 56 1,22,3,24,4,25,5,23" "256 64 1 1 56 1,22,4,25" "128 128 3 1 28 1,22,3,24,5,23" "256 256 3 1 14 1,22,3,24,5,23" "512 512 3 1 7 1,22,5,23" "1024 256 1 1 14 1,22,5,23" "512 2048 1 1 7 1,22,5,23"; do
  timeout -k 10 120 python scripts/conv_time.py $spec --stats 2>&1 | grep -v amdgpu.ids || exit 1
done
bash scripts/archive/gpu_ab_env.sh DAMD_CONV_EXCLUDE "*:22-25" ""
