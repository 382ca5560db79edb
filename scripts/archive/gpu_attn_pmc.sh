#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
rm -rf gpurun_out/pmc_a gpurun_out/pmc_b
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU -d gpurun_out/pmc_a -o run --output-format csv -- python scripts/archive/attn_fwd_only.py bwd > gpurun_out/pmc_a.log 2>&1 || { tail -5 gpurun_out/pmc_a.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc_b -o run --output-format csv -- python scripts/archive/attn_fwd_only.py bwd > gpurun_out/pmc_b.log 2>&1 || { tail -5 gpurun_out/pmc_b.log; exit 1; }
find gpurun_out/pmc_a gpurun_out/pmc_b -name "*counter_collection.csv" | head
