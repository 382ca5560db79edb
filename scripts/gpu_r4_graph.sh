#!/bin/bash
# Device-side dropout seeds + whole-step hipGraph capture: attention / norm dropout tests, graph tests, BERT throughput.
source "$(dirname "$0")/gpu_lib.sh"
PYT="python -u -m pytest -x -v --timeout-method thread"
step graph_tests 400 $PYT --timeout 180 tests/test_attention_mask_dropout_gpu.py tests/test_attention_gpu.py tests/test_graphs_gpu.py tests/test_ops_gpu.py
[ $status -ne 0 ] && exit 1
step bert_bench 400 python -u scripts/bert_bench.py --batch 64 --seq 128 --steps 30 --warmup 10
exit $status
