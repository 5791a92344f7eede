#!/bin/bash
# Pass B tiles dealt to the XCDs in contiguous runs (exp/bxcd) vs the default, alternating.
set -o pipefail
TAG=${1:-r02bx}
mkdir -p gpurun_out
L="--steps 10 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline"
timeout -k 10 200 python -u bench.py $L > gpurun_out/${TAG}_def.log 2>&1 || exit $?
COMAP_HIP_LIB=$PWD/exp/bxcd/libcomap_hip.so timeout -k 10 300 python -u bench.py $L --check > gpurun_out/${TAG}_bxcd.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py $L > gpurun_out/${TAG}_def2.log 2>&1 || exit $?
COMAP_HIP_LIB=$PWD/exp/bxcd/libcomap_hip.so timeout -k 10 300 python -u bench.py $L > gpurun_out/${TAG}_bxcd2.log 2>&1 || exit $?
COMAP_HIP_LIB=$PWD/exp/bxcd/libcomap_hip.so timeout -k 10 300 python -u bench.py $L --shard-of 8 > gpurun_out/${TAG}_bxcd_s8.log 2>&1 || exit $?
