#!/bin/bash
# Steady-state kernel profile of the headline ResNet-50 bench (in-tree MIOpen find-db).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
BATCH=${1:-512}
rm -rf gpurun_out/prof_r
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r -o run --output-format csv -- python bench.py --steps 8 --warmup 4 --batch $BATCH > gpurun_out/prof_r.log 2>&1
rc=$?; echo "rocprof exit $rc"; tail -2 gpurun_out/prof_r.log
[ $rc -ne 0 ] && exit 1
f=$(find gpurun_out/prof_r -name "*kernel_trace.csv" | head -1)
python scripts/prof_steady.py "$f" --steps 6 --top 45 --seq gpurun_out/prof_r_seq.txt > gpurun_out/prof_r_summary.txt && cat gpurun_out/prof_r_summary.txt | head -70
rm -f "$f"
