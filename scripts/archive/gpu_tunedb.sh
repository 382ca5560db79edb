#!/bin/bash
# Generate the in-tree conv tuning database (per-layer kernel choices at batch 512), then time the
# bench starting from it vs tuning from scratch (same box).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
DAMD_CONV_TUNE_DB="" timeout -k 10 400 python bench.py --steps 20 --warmup 6 --save-tune-db gpurun_out/conv_tune_db.jsonl > gpurun_out/tdb_gen.log 2>&1 || { tail -20 gpurun_out/tdb_gen.log; exit 1; }
echo "tuned from scratch: $(grep 'warmup 6/6' gpurun_out/tdb_gen.log) $(tail -1 gpurun_out/tdb_gen.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
DAMD_CONV_TUNE_DB=gpurun_out/conv_tune_db.jsonl timeout -k 10 400 python bench.py --steps 30 --warmup 6 > gpurun_out/tdb_use.log 2>&1 || { tail -20 gpurun_out/tdb_use.log; exit 1; }
echo "from the db: $(grep 'warmup 6/6' gpurun_out/tdb_use.log) $(tail -1 gpurun_out/tdb_use.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
