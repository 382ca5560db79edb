#!/bin/bash
# Same-box A/B: bench starting from the in-tree tuning database vs tuning from scratch, interleaved.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/tdb_ab.txt
for db in default none default none; do
  if [ "$db" = none ]; then export DAMD_CONV_TUNE_DB=""; else unset DAMD_CONV_TUNE_DB; fi
  timeout -k 10 400 python bench.py --steps 30 --warmup 6 > gpurun_out/tdb.log 2>&1 || { tail -20 gpurun_out/tdb.log; exit 1; }
  echo "db=$db $(grep 'warmup 6/6' gpurun_out/tdb.log) $(tail -1 gpurun_out/tdb.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')" | tee -a gpurun_out/tdb_ab.txt
done
