#!/bin/bash
# Same-box A/B of MIOpen find-db rankings (in-tree db vs CK-preferred backward-data variants).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/db_ab.jsonl; : > $out
python scripts/miopen_db_prefer_ck.py determined_amd/benchmarks/miopen_db gpurun_out/db_ck10 --margin 0.10 || exit 1
python scripts/miopen_db_prefer_ck.py determined_amd/benchmarks/miopen_db gpurun_out/db_ck25 --margin 0.25 || exit 1
for db in determined_amd/benchmarks/miopen_db gpurun_out/db_ck10 gpurun_out/db_ck25 determined_amd/benchmarks/miopen_db; do
  MIOPEN_USER_DB_PATH=$PWD/$db timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/db_one.log 2>&1 || { echo "bench failed ($db)"; tail -5 gpurun_out/db_one.log; exit 1; }
  v=$(tail -1 gpurun_out/db_one.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
  echo "{\"db\": \"$db\", \"samples_per_s\": $v}" | tee -a $out
done
