#!/bin/bash
# Destriper projection grid: parity tests, then C4/C5 legs with the fixed 1024-block cap vs the budgeted cap.
set -o pipefail
TAG=${1:-r02pg}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_destriper.py tests/test_gpu_c2.py tests/test_mapmaking_driver.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || exit $?
B="--steps 1 --warmup 1 --no-cpu-baseline --no-e2e"
COMAP_DS_PROJ_BUDGET=0 timeout -k 10 300 python -u bench.py $B > gpurun_out/${TAG}_b0.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py $B > gpurun_out/${TAG}_bdef.log 2>&1 || exit $?
