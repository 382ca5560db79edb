#!/bin/bash
# hipBLASLt GEMM candidate for the 1x1 weight gradient: test, then a same-box A/B in the headline bench.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step g1_tests 300 $PYT --timeout 120 tests/test_conv_gpu.py -k "gemm_candidate"
[ $status -ne 0 ] && exit 1
out=gpurun_out/ab_gemm.jsonl; : > $out
i=0
for ex in "" "wgrad:gemm" "" "wgrad:gemm"; do
  i=$((i+1))
  export DAMD_CONV_EXCLUDE="$ex"
  step abg$i 300 python bench.py --steps 20 --warmup 5
  v=$(tail -1 gpurun_out/abg$i.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])") || exit 1
  echo "{\"excluded\": \"$ex\", \"samples_per_s\": $v}" | tee -a $out
done
exit $status
