#!/bin/bash
# C3 rank-0 shard: wavelet-matrix segment target sweep (the C2 plan is cap-driven, see median_kernels.hip)
set -o pipefail
TAG=${1:-r02sw2}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-destriper --no-e2e --shard-of 8"
for s in 1 64 128 192 256; do
  COMAP_MEDIAN_WMSEGS=$s timeout -k 10 200 $B > gpurun_out/${TAG}_wm$s.log 2>&1 || exit $?
done
COMAP_MEDIAN_WMSEGS=128 timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-destriper --no-e2e > gpurun_out/${TAG}_c2_wm128.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-destriper --no-e2e > gpurun_out/${TAG}_c2_wm256.log 2>&1 || exit $?
