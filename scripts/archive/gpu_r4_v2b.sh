#!/bin/bash
# conv3x3v2 without the scratch-resident halo registers: correctness, per-config timing at the bench
# batch, BERT tests, then the headline bench and its steady-state profile.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step v2_tests 240 $PYT --timeout 120 tests/test_conv3x3v2_gpu.py
step v2_bench 300 python -u scripts/v2_bench.py --batch 2048 --out gpurun_out/v2_bench2.jsonl
step bert_tests 240 $PYT --timeout 200 tests/test_bert_gpu.py
step bench 300 python bench.py --steps 20 --warmup 5
step prof_resnet 420 bash scripts/gpu_prof_resnet.sh 2048
exit $status
