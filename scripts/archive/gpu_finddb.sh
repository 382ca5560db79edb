#!/bin/bash
# Populate MIOpen's find-db for the ResNet-50 convolutions MIOpen still runs at a new per-GPU batch
# (cudnn.benchmark search), into gpurun_out/miopen_db_new (merged back; copied in-tree afterwards).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/miopen_db_new
cp determined_amd/benchmarks/miopen_db/*.txt gpurun_out/miopen_db_new/ 2>/dev/null
export HSA_ENABLE_IPC_MODE_LEGACY=0 MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db_new
timeout -k 10 1080 python bench.py --batch ${1:-2048} --steps 3 --warmup 2 > gpurun_out/finddb.log 2>&1 || { echo "bench failed/timed out"; grep -v "warming up" gpurun_out/finddb.log | tail -5; ls -la gpurun_out/miopen_db_new; exit 1; }
tail -1 gpurun_out/finddb.log
ls -la gpurun_out/miopen_db_new
