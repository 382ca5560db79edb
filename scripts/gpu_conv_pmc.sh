#!/bin/bash
# PMC passes over single conv configs: scripts/gpu_conv_pmc.sh "CIN COUT K S HW CFG" ...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
i=0
for spec in "$@"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_c$i
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU -d gpurun_out/pmc_c$i/a -o run --output-format csv -- python scripts/conv_one.py $spec > gpurun_out/pmc_c$i.log 2>&1 || { tail -5 gpurun_out/pmc_c$i.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc_c$i/b -o run --output-format csv -- python scripts/conv_one.py $spec >> gpurun_out/pmc_c$i.log 2>&1 || { tail -5 gpurun_out/pmc_c$i.log; exit 1; }
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_c$i/t -o run --output-format csv -- python scripts/conv_one.py $spec >> gpurun_out/pmc_c$i.log 2>&1 || { tail -5 gpurun_out/pmc_c$i.log; exit 1; }
done
python3 - "$@" <<'PY'
import csv, glob, sys
for i, spec in enumerate(sys.argv[1:], 1):
    vals = {}
    for part in ("a", "b"):
        for f in glob.glob(f"gpurun_out/pmc_c{i}/{part}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "conv" not in r.get("Kernel_Name", ""):
                    continue
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    dur = []
    for f in glob.glob(f"gpurun_out/pmc_c{i}/t/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "conv" in r["Name"]:
                dur.append(float(r["AverageNs"]) / 1e3)
    agg = {k: sum(v) / max(1, len(v)) for k, v in vals.items()}
    print(spec, "avg_us", [round(d, 1) for d in dur])
    for k in sorted(agg):
        print(f"   {k:28s} {agg[k]:.4g}")
PY
