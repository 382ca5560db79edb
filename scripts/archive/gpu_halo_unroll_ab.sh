#!/bin/bash
# 3x3 halo kernel with the 9-tap unrolled unit body vs determined_amd/ops/ref (previous build):
# conv GPU tests + end-to-end training parity on the new build, halo per-config times at batch 2048
# (forward + stats, BN-apply prologue forward, deferred-BN-backward input gradient), then an
# interleaved headline-bench A/B at the default batch on one box.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
REF=$PWD/determined_amd/ops/ref/_hip_ops.cpython-310-x86_64-linux-gnu.so
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_ops_gpu.py tests/test_resnet_training_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/hu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/hu_tests.log; exit 1; }
tail -1 gpurun_out/hu_tests.log
for lib in new ref; do
  if [ $lib = ref ]; then export DAMD_HIP_OPS_PATH=$REF; else unset DAMD_HIP_OPS_PATH; fi
  HALO_BATCH=2048 timeout -k 10 300 python scripts/archive/halo_ws_time.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$lib /" | tee -a gpurun_out/hu_time.txt || exit 1
done
for lib in ref new ref new; do
  if [ $lib = ref ]; then export DAMD_HIP_OPS_PATH=$REF; else unset DAMD_HIP_OPS_PATH; fi
  timeout -k 10 400 python bench.py --steps 12 --warmup 4 > gpurun_out/hu_ab.log 2>&1 || { tail -20 gpurun_out/hu_ab.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/hu_ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/hu_ab_summary.txt
done
