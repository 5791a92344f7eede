#!/bin/bash
# GPU suite (vane on the side stream), L1 bench with/without the side-stream vane, file -> HBM staging
# with the pread direct path, C3 shard-of-8 median segment sweep.
set -o pipefail
TAG=${1:-r02h5b}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || exit $?
L="--steps 10 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline"
timeout -k 10 200 python -u bench.py $L > gpurun_out/${TAG}_l1_side.log 2>&1 || exit $?
COMAP_VANE_SIDE=0 timeout -k 10 200 python -u bench.py $L > gpurun_out/${TAG}_l1_main.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/h5_upload.py 2 180000 > gpurun_out/${TAG}_upload.log 2>&1 || exit $?
for m in 0 220 440 880; do
  COMAP_MEDIAN_MINSEGS=$m timeout -k 10 200 python -u bench.py $L --shard-of 8 > gpurun_out/${TAG}_ms$m.log 2>&1 || exit $?
done
