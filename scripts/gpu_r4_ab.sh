#!/bin/bash
# Same-box A/B of the conv3x3v2 configs in the headline bench (box-to-box spread is ~2%): all configs,
# without the resident-filter config (32), without any conv3x3v2 config (26-32), all again.
source "$(dirname "$0")/gpu_lib.sh"
out=gpurun_out/ab_v2.jsonl; : > $out
i=0
for ex in "" "*:32" "*:26-32" ""; do
  i=$((i+1))
  export DAMD_CONV_EXCLUDE="$ex"
  step ab$i 300 python bench.py --steps 20 --warmup 5
  v=$(tail -1 gpurun_out/ab$i.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])") || exit 1
  echo "{\"excluded\": \"$ex\", \"samples_per_s\": $v}" | tee -a $out
done
exit $status
