#!/bin/bash
# Multi-rank CG with block partials all-reduced (4 launches): destriper GPU tests (incl. uneven 2-rank
# split), the multi-rank driver's cost on one rank vs the native solve, and the 2-rank self-launched bench.
set -o pipefail
TAG=${1:-r02df}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_destriper.py tests/test_mapmaking_driver.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || exit $?
for a in "1 1" "1 4" "8 1" "8 4"; do
  timeout -k 10 200 python -u scripts/ds_eager.py $a 96 >> gpurun_out/${TAG}_eager.log 2>&1 || exit $?
done
COMAP_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 --feeds 6 --no-cpu-baseline --c5-obs 2 --no-e2e > gpurun_out/${TAG}_2rank.log 2>&1 || exit $?
