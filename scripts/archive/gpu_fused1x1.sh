#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_bn_gpu.py -x -q --timeout 200 --timeout-method thread -k "bwd_fused or chained or resnet50_bf16 or bottleneck" > gpurun_out/f1_tests.log 2>&1 || { tail -40 gpurun_out/f1_tests.log; exit 1; }
tail -1 gpurun_out/f1_tests.log
rm -f gpurun_out/ab_summary.txt gpurun_out/tune_choices.txt
for ex in "" "bwd1x1_fused:0"; do
  DAMD_CONV_EXCLUDE="$ex" DAMD_TUNE_DUMP=gpurun_out/tune_choices.txt timeout -k 10 400 python bench.py --steps 30 --warmup 6 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  echo "exclude=[$ex] $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/ab_summary.txt
done
grep bwd1x1 gpurun_out/tune_choices.txt | head -4
