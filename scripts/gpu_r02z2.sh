#!/bin/bash
# pass A variants: aligned DPP kernel with 3/4 groups at occupancy 2; unaligned 2 rows x 8 groups (occupancy 4)
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline"
for v in vC vD; do
  COMAP_HIP_LIB=$PWD/exp/$v/libcomap_hip.so timeout -k 10 200 python -u bench.py $B > gpurun_out/r02z2_$v.log 2>&1 || exit $?
done
COMAP_A_DPP=0 COMAP_HIP_LIB=$PWD/exp/vE/libcomap_hip.so timeout -k 10 200 python -u bench.py $B > gpurun_out/r02z2_vE.log 2>&1 || exit $?
