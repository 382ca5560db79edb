#!/bin/bash
# Same-box A/B of the conv3x3v2 weight gradient in the headline bench; BERT bf16-weights test + throughput.
source "$(dirname "$0")/gpu_lib.sh"
out=gpurun_out/ab_w.jsonl; : > $out
i=0
for ex in "" "wgrad:h2,wgrad:h3,wgrad:h4" ""; do
  i=$((i+1))
  export DAMD_CONV_EXCLUDE="$ex"
  step abw$i 300 python bench.py --steps 20 --warmup 5
  v=$(tail -1 gpurun_out/abw$i.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])") || exit 1
  echo "{\"excluded\": \"$ex\", \"samples_per_s\": $v}" | tee -a $out
done
unset DAMD_CONV_EXCLUDE
PYT="python -u -m pytest -x -v --timeout-method thread"
step bert_tests 400 $PYT --timeout 300 tests/test_bert_gpu.py -k follows_fp32
step bert_bench 300 python -u scripts/bert_bench.py --batch 64 --seq 128 --steps 30 --warmup 10
exit $status
