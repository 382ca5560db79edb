#!/bin/bash
# Round 3: gradient-parity diagnostics, the hooked-conv test, then rehearsal + layer roofline.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rw in 0.2 1.0; do
  RES_W=$rw timeout -k 10 300 python scripts/dev/grad_parity.py > gpurun_out/grad_parity_$rw.log 2>&1 || { echo "parity $rw failed"; tail -20 gpurun_out/grad_parity_$rw.log; exit 1; }
  tail -7 gpurun_out/grad_parity_$rw.log
done
bash scripts/archive/gpu_r3a.sh
