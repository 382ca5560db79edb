#!/bin/bash
# Round 3: round-end rehearsal (GPU tests, smoke, bench) + per-layer roofline table at batch 1024.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_roundend.sh || exit 1
timeout -k 10 400 python scripts/layer_roofline.py --batch 1024 > gpurun_out/layer_roofline.log 2>&1 || { echo "roofline failed"; tail -20 gpurun_out/layer_roofline.log; exit 1; }
tail -3 gpurun_out/layer_roofline.log
