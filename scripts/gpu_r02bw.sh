#!/bin/bash
# pass B at 3 waves per SIMD (COMAP_B_WPE=3; 2 or 1 channel rows per load batch) vs the default 2
set -o pipefail
TAG=${1:-r02bw}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-destriper --no-e2e"
timeout -k 10 200 $B > gpurun_out/${TAG}_def.log 2>&1 || exit $?
for v in w3 w3b1; do
  COMAP_HIP_LIB=$PWD/exp/$v/libcomap_hip.so timeout -k 10 200 $B > gpurun_out/${TAG}_$v.log 2>&1 || exit $?
done
timeout -k 10 200 $B > gpurun_out/${TAG}_def2.log 2>&1 || exit $?
