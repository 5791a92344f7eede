#!/bin/bash
# Multi-rank CG driver with its pieces bound once: parity, then host cost vs the native solve.
set -o pipefail
TAG=${1:-r02eg}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_destriper.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || exit $?
for a in "1 1" "1 4" "8 1" "8 4"; do
  timeout -k 10 200 python -u scripts/ds_eager.py $a 96 >> gpurun_out/${TAG}_eager.log 2>&1 || exit $?
done
