#!/bin/bash
# CG bin over compacted hit-row ranges: destriper parity (small, C4, C5) and the C4/C5 bench legs.
set -o pipefail
TAG=${1:-r02hp}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_destriper.py tests/test_gpu_c2.py tests/test_mapmaking_driver.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
