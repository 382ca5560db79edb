#!/bin/bash
# Wave-specialised 3x3 halo configs: GPU correctness tests, per-layer timing, then a same-box
# interleaved A/B of the headline bench with configs 26-28 excluded vs included.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_ops_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "conv" > gpurun_out/ws_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ws_tests.log; exit 1; }
tail -1 gpurun_out/ws_tests.log
timeout -k 10 300 python scripts/archive/halo_ws_time.py > gpurun_out/ws_time.jsonl 2>&1 || { echo "timing failed"; tail -20 gpurun_out/ws_time.jsonl; exit 1; }
cat gpurun_out/ws_time.jsonl
for ex in "*:26-28" "" "*:26-28" ""; do
  DAMD_CONV_EXCLUDE="$ex" timeout -k 10 400 python bench.py --steps 30 --warmup 8 > gpurun_out/ws_ab.log 2>&1 || { tail -20 gpurun_out/ws_ab.log; exit 1; }
  echo "exclude=[$ex] $(tail -1 gpurun_out/ws_ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a gpurun_out/ws_ab_summary.txt
done
bash scripts/archive/gpu_multirank_rehearsal.sh
