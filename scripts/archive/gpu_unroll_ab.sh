#!/bin/bash
# Conv kernel A/B: the current build vs determined_amd/ops/ref (previous conv_igemm.hip, same other
# kernels): conv GPU tests + end-to-end training parity on the new build, per-layer times, then an
# interleaved headline-bench A/B at batch 2048 on one box.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
REF=$PWD/determined_amd/ops/ref/_hip_ops.cpython-310-x86_64-linux-gnu.so
BUF=$PWD/determined_amd/ops/buf/_hip_ops.cpython-310-x86_64-linux-gnu.so
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_ops_gpu.py tests/test_resnet_training_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/ua_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ua_tests.log; exit 1; }
tail -1 gpurun_out/ua_tests.log
for lib in new ref buf; do
  if [ $lib = ref ]; then export DAMD_HIP_OPS_PATH=$REF; elif [ $lib = buf ]; then export DAMD_HIP_OPS_PATH=$BUF; else unset DAMD_HIP_OPS_PATH; fi
  for spec in "256 256 3 1 14 12,22" "128 128 3 1 28 12,22" "64 256 1 1 56 13" "256 64 1 1 56 4" "1024 256 1 1 14 13" "512 512 3 1 7 12,14"; do
    timeout -k 10 120 python scripts/conv_time.py $spec --batch 2048 2>&1 | grep -v amdgpu | sed "s/^/$lib /" | tee -a gpurun_out/ua_layers.txt
  done
done
unset DAMD_HIP_OPS_PATH
for lib in ref new buf new; do
  if [ $lib = ref ]; then export DAMD_HIP_OPS_PATH=$REF; elif [ $lib = buf ]; then export DAMD_HIP_OPS_PATH=$BUF; else unset DAMD_HIP_OPS_PATH; fi
  timeout -k 10 400 python bench.py --batch 2048 --steps 12 --warmup 4 --conv-benchmark 0 > gpurun_out/ua_ab.log 2>&1 || { tail -20 gpurun_out/ua_ab.log; exit 1; }
  echo "$lib $(tail -1 gpurun_out/ua_ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/ua_ab_summary.txt
done
