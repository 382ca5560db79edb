#!/bin/bash
# Multi-rank rehearsal at the bench batch (2 torchrun ranks on the GPU over gloo: JSON contract,
# tuning time) and the GPT-2 345M ZeRO-2 number + steady-state profile on the current build.
source "$(dirname "$0")/gpu_lib.sh"
step multirank 600 bash scripts/gpu_multirank_b2048.sh
grep -E "tuned|warmup 1/" gpurun_out/mr2k.err | head -4
step gpt2_bench 400 python -m determined_amd.benchmarks.gpt2 --mb 8 --steps 10 --warmup 3
step prof_gpt2 450 bash scripts/gpu_prof_gpt2.sh
exit $status
