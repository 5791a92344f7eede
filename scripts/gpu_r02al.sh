#!/bin/bash
# aligned pass A (COMAP_A_DPP=1) with the airmass staged through LDS (COMAP_A_ALDS=1; DPP or
# second-load pair sample; 2 or 4 chunk groups) vs the default k_moments; then parity of each
set -o pipefail
TAG=${1:-r02al}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-destriper --no-e2e"
timeout -k 10 200 $B > gpurun_out/${TAG}_def.log 2>&1 || exit $?
for v in alds aldsx alds4; do
  COMAP_A_DPP=1 COMAP_HIP_LIB=$PWD/exp/$v/libcomap_hip.so timeout -k 10 200 $B > gpurun_out/${TAG}_$v.log 2>&1 || exit $?
done
timeout -k 10 200 $B > gpurun_out/${TAG}_def2.log 2>&1 || exit $?
for v in alds aldsx alds4; do
  COMAP_A_DPP=1 COMAP_HIP_LIB=$PWD/exp/$v/libcomap_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_l1.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest_$v.log 2>&1 || exit $?
done
