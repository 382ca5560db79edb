#!/bin/bash
# 3x3 halo prologues: GPU tests, then a same-box A/B of the headline bench with / without them.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_conv_gpu.py tests/test_bn_gpu.py -x -q --timeout 200 --timeout-method thread -k "halo_prologue or bnact or dgrad or bottleneck or chained or resnet" > gpurun_out/pro3_tests.log 2>&1 || { tail -40 gpurun_out/pro3_tests.log; exit 1; }
tail -1 gpurun_out/pro3_tests.log
rm -f gpurun_out/ab_summary.txt
for ex in "" "fwd_pro:7,fwd_pro:19,dgrad_bn_pro:7,dgrad_bn_pro:19"; do
  DAMD_CONV_EXCLUDE="$ex" DAMD_TUNE_DUMP=gpurun_out/tune_choices.txt timeout -k 10 400 python bench.py --steps 30 --warmup 8 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  echo "exclude=[$ex] $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/ab_summary.txt
done
