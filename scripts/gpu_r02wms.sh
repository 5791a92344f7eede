#!/bin/bash
# Wavelet-matrix segment target at a C3 shard (110 series) and at C2 (836 series).
set -o pipefail
TAG=${1:-r02wms}
mkdir -p gpurun_out
L="--steps 10 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline"
for s in 128 256 384 512; do
  COMAP_MEDIAN_WMSEGS=$s timeout -k 10 200 python -u bench.py $L --shard-of 8 > gpurun_out/${TAG}_s8_$s.log 2>&1 || exit $?
done
for s in 256 512 1024 2048; do
  COMAP_MEDIAN_WMSEGS=$s timeout -k 10 200 python -u bench.py $L > gpurun_out/${TAG}_c2_$s.log 2>&1 || exit $?
done
