#!/bin/bash
# LDS-staged airmass (pass A) + median filter (pass C): parity, A/B vs default
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/exp/ac1/libcomap_hip.so
COMAP_HIP_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_l1.py -m gpu -x -q --timeout 200 --timeout-method thread -k "residues or multi_feed or c1 or averaged or atmosphere or edge_variants or shards" > gpurun_out/r02ac_pytest.log 2>&1 || exit $?
B="--steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline"
timeout -k 10 200 python -u bench.py $B > gpurun_out/r02ac_base.log 2>&1 || exit $?
COMAP_HIP_LIB=$L timeout -k 10 200 python -u bench.py $B --check > gpurun_out/r02ac_ac1.log 2>&1 || exit $?
COMAP_HIP_LIB=$PWD/exp/ac4/libcomap_hip.so timeout -k 10 200 python -u bench.py $B > gpurun_out/r02ac_ac4.log 2>&1 || exit $?
