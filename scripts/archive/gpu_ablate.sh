#!/bin/bash
# A/B of the ResNet-50 model-level fusions on ONE box (box-to-box variance is a few %):
# each line is bench.py with DAMD_DISABLE_FUSIONS set as labelled.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/ablate.jsonl; : > $out
for dis in "" "stem_conv" "stem_stats" "split_grad" "avgpool" "stem_conv,split_grad,avgpool" ""; do
  DAMD_DISABLE_FUSIONS="$dis" timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/ablate_one.log 2>&1 || { echo "bench failed ($dis)"; tail -5 gpurun_out/ablate_one.log; exit 1; }
  v=$(tail -1 gpurun_out/ablate_one.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
  echo "{\"disabled\": \"$dis\", \"samples_per_s\": $v}" | tee -a $out
done
