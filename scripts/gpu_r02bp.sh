#!/bin/bash
# Pass B with the channel ids loaded one batch ahead (exp/bpref: 2 rows per batch, exp/bpref3: 3), vs the default.
set -o pipefail
TAG=${1:-r02bp}
mkdir -p gpurun_out
L="--steps 10 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline"
timeout -k 10 200 python -u bench.py $L > gpurun_out/${TAG}_def.log 2>&1 || exit $?
for v in bpref bpref3; do
  COMAP_HIP_LIB=$PWD/exp/$v/libcomap_hip.so timeout -k 10 300 python -u bench.py $L --check > gpurun_out/${TAG}_$v.log 2>&1 || exit $?
done
timeout -k 10 200 python -u bench.py $L > gpurun_out/${TAG}_def2.log 2>&1 || exit $?
