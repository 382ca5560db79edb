#!/bin/bash
# 3x3 halo conv kernel A/B (DAMD_HALO_SCH=0 vs 1, same box, interleaved): numerics tests under the
# new schedule, then per-config timings on the ResNet-50 3x3 shapes (batch 1024).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
DAMD_HALO_SCH=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > gpurun_out/halo_tests.log 2>&1 || { echo "conv tests failed"; tail -30 gpurun_out/halo_tests.log; exit 1; }
tail -1 gpurun_out/halo_tests.log
for rep in 1 2; do
for sch in 0 1; do
for spec in "64 64 3 1 56 7,19" "128 128 3 1 28 6,18,19" "256 256 3 1 14 6,9,18" "512 512 3 1 7 9,18,21"; do
  DAMD_HALO_SCH=$sch timeout -k 10 120 python scripts/conv_time.py $spec --stats 2>&1 | grep -v amdgpu.ids | sed "s/^/sch$sch /" || exit 1
done
done
done
