#!/bin/bash
# pass A wave shapes: rows per wave (COMAP_CPW) x sample groups per trip (COMAP_AUNR) vs the default 4 x 4
set -o pipefail
TAG=${1:-r02av}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-destriper --no-e2e"
timeout -k 10 200 $B > gpurun_out/${TAG}_def.log 2>&1 || exit $?
for v in a8u2 a2u4 a2u8; do
  COMAP_HIP_LIB=$PWD/exp/$v/libcomap_hip.so timeout -k 10 200 $B > gpurun_out/${TAG}_$v.log 2>&1 || exit $?
done
