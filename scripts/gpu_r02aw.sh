#!/bin/bash
# pass A at 4 waves per SIMD (COMAP_AM_WPE=4: 128 VGPRs, 48 B/lane spill) vs the default 3
set -o pipefail
TAG=${1:-r02aw}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-destriper --no-e2e"
timeout -k 10 200 $B > gpurun_out/${TAG}_def.log 2>&1 || exit $?
COMAP_HIP_LIB=$PWD/exp/am4/libcomap_hip.so timeout -k 10 200 $B > gpurun_out/${TAG}_am4.log 2>&1 || exit $?
timeout -k 10 200 $B > gpurun_out/${TAG}_def2.log 2>&1 || exit $?
