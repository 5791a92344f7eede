#!/bin/bash
# Wavelet-matrix walk with 2 (default) / 1 / 4 outputs per thread walking the levels together.
set -o pipefail
TAG=${1:-r02wqq}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_l1.py -x -q -m gpu --timeout 300 --timeout-method thread -k "medfilt or median or c1" > gpurun_out/${TAG}_pytest.log 2>&1 || exit $?
L="--steps 10 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline"
timeout -k 10 200 python -u bench.py $L > gpurun_out/${TAG}_q2.log 2>&1 || exit $?
COMAP_HIP_LIB=$PWD/exp/wq1/libcomap_hip.so timeout -k 10 200 python -u bench.py $L > gpurun_out/${TAG}_q1.log 2>&1 || exit $?
COMAP_HIP_LIB=$PWD/exp/wq4/libcomap_hip.so timeout -k 10 200 python -u bench.py $L > gpurun_out/${TAG}_q4.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py $L --shard-of 8 > gpurun_out/${TAG}_q2_s8.log 2>&1 || exit $?
COMAP_HIP_LIB=$PWD/exp/wq1/libcomap_hip.so timeout -k 10 200 python -u bench.py $L --shard-of 8 > gpurun_out/${TAG}_q1_s8.log 2>&1 || exit $?
COMAP_HIP_LIB=$PWD/exp/wq4/libcomap_hip.so timeout -k 10 200 python -u bench.py $L --shard-of 8 > gpurun_out/${TAG}_q4_s8.log 2>&1 || exit $?
