#!/bin/bash
# Round-4 kernels on the GPU: conv3x3v2 vs fp32, attention key-padding / dropout, DDP over the fused
# ResNet-50 (2 gloo ranks), BERT-base MLM (HF Trainer + DetCallback), then per-config timing of the
# 3x3 layers at the bench batch.  A failing test does not stop the run; a fault, abort, segfault or
# time-out does (nothing more is started on the GPU after one).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
status=0

step() {  # step <name> <timeout> <cmd...>
  local name=$1 limit=$2
  shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || grep -q "+++++++ Timeout +++++++" "gpurun_out/$name.log"; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
  [ $rc -ne 0 ] && status=1
  return 0
}

PYT="python -u -m pytest -x -v --timeout-method thread"
step v2_tests 300 $PYT --timeout 120 tests/test_conv3x3v2_gpu.py
step attn_tests 300 $PYT --timeout 120 tests/test_attention_mask_dropout_gpu.py tests/test_attention_gpu.py
step ddp_test 330 $PYT --timeout 300 tests/test_ddp_fused_gpu.py
step bert_tests 400 $PYT --timeout 300 tests/test_bert_gpu.py
step v2_bench 500 python -u scripts/v2_bench.py --batch 2048 --out gpurun_out/v2_bench.jsonl
cat gpurun_out/v2_bench.jsonl
exit $status
