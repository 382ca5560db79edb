#!/bin/bash
# Kernel times + SQ counters of the fused stem kernels (scripts/stem_time.py at batch 1024).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp PYTHONPATH=$PWD
rm -rf gpurun_out/stem_prof gpurun_out/stem_pmc*
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stem_prof -o run --output-format csv -- python scripts/stem_time.py --iters 3 > gpurun_out/stem_prof.log 2>&1 || { tail -20 gpurun_out/stem_prof.log; exit 1; }
f=$(find gpurun_out/stem_prof -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us x{r["Calls"]:>3}  {r["Name"][:110]}')
PY
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/stem_pmc$i -o run --output-format csv -- python scripts/stem_time.py --iters 1 > gpurun_out/stem_pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/stem_pmc$i.log; exit 1; }
  f=$(find gpurun_out/stem_pmc$i -name "*counter_collection.csv" | head -1)
  python - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"]
    if "stem" not in k and "maxpool" not in k and "pooled" not in k: continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k[:90]); print("   " + "  ".join(f"{c}={v:.3g}" for c, v in sorted(d.items())))
PY
done
