#!/bin/bash
# Round-3 re-entry check: full GPU tests, smoke, fused-stem kernel timing, then a same-box
# interleaved A/B of the headline bench with the fused stem off vs on.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3d_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r3d_pytest.log; exit 1; }
tail -1 gpurun_out/r3d_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3d_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r3d_smoke.log; exit 1; }
tail -1 gpurun_out/r3d_smoke.log
timeout -k 10 200 python scripts/stem_time.py --iters 10 > gpurun_out/r3d_stem.log 2>&1 || { echo "stem_time failed"; tail -20 gpurun_out/r3d_stem.log; exit 1; }
tail -1 gpurun_out/r3d_stem.log
bash scripts/archive/gpu_ab_fusion.sh "" stem_pool
