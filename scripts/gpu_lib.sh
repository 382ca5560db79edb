# Sourced by the gpu_*.sh wrappers: run one GPU step under its own time limit; a failing step
# marks the run failed but the next one still runs, while a fault / abort / segfault / time-out
# (exit >= 124, or a pytest-timeout dump) ends the script: nothing more starts on the GPU after it.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
status=0

step() {  # step <name> <timeout-seconds> <cmd...>  (stdout+stderr -> gpurun_out/<name>.log)
  local name=$1 limit=$2
  shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || grep -q "+++++++ Timeout +++++++" "gpurun_out/$name.log"; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
  [ $rc -ne 0 ] && status=1
  return 0
}
