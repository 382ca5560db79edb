#!/bin/bash
# Same-box A/B: per-layer timed 1x1 BN prologues (default) vs always-fused 1x1 prologues (DAMD_PRO_ALWAYS_1X1=1,
# no standalone BN apply passes before 1x1 convs); then a steady-state profile at batch 256.
source "$(dirname "$0")/gpu_lib.sh"
out=gpurun_out/ab_pro.jsonl; : > $out
i=0
for pa in 0 1 0 1; do
  i=$((i+1))
  export DAMD_PRO_ALWAYS_1X1=$pa
  step abp$i 300 python bench.py --steps 20 --warmup 5
  v=$(tail -1 gpurun_out/abp$i.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])") || exit 1
  echo "{\"DAMD_PRO_ALWAYS_1X1\": $pa, \"samples_per_s\": $v}" | tee -a $out
done
unset DAMD_PRO_ALWAYS_1X1
step prof256 300 bash scripts/gpu_prof_resnet.sh 256
cp gpurun_out/prof_r_summary.txt gpurun_out/prof_r256_summary.txt
exit $status
