#!/bin/bash
# Lazy-direction CG: bit-identity vs the 4-launch CG, destriper parity (small, C4, C5), C4/C5 legs both ways.
set -o pipefail
TAG=${1:-r02ld}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_destriper.py tests/test_gpu_c2.py tests/test_mapmaking_driver.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || exit $?
B="--steps 1 --warmup 1 --no-cpu-baseline --no-e2e"
COMAP_DS_LAZY=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/${TAG}_b0.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py $B > gpurun_out/${TAG}_bdef.log 2>&1 || exit $?
COMAP_DS_LAZY=1 timeout -k 10 300 python -u bench.py $B > gpurun_out/${TAG}_b1.log 2>&1 || exit $?
