set -o pipefail
cd /root/repo
export PYTHONPATH=$PWD
for lib in new ref; do
  if [ $lib = ref ]; then export DAMD_HIP_OPS_PATH=$PWD/determined_amd/ops/ref/_hip_ops.cpython-310-x86_64-linux-gnu.so; else unset DAMD_HIP_OPS_PATH; fi
  for spec in "64 256 1 1 56 13" "256 64 1 1 56 4,13" "64 64 3 1 56 7,12"; do
    timeout -k 10 120 python scripts/conv_time.py $spec --batch 2048 2>&1 | sed "s/^/$lib /"
  done
done
