#!/bin/bash
# C3 rank-0 shard (8-way split of C2) on one GPU: default vs the side-stream vane,
# the 2-group pass B / median / pass C pipeline and fewer wavelet-matrix segments,
# which may pay at shard size where the median and vane are a larger share.
set -o pipefail
TAG=${1:-r02sw}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-destriper --no-e2e --shard-of 8"
timeout -k 10 200 $B > gpurun_out/${TAG}_default.log 2>&1 || exit $?
COMAP_VANE_SIDE=1 timeout -k 10 200 $B > gpurun_out/${TAG}_vaneside.log 2>&1 || exit $?
COMAP_GROUPS=2 timeout -k 10 200 $B > gpurun_out/${TAG}_groups2.log 2>&1 || exit $?
COMAP_MEDIAN_WMSEGS=128 timeout -k 10 200 $B > gpurun_out/${TAG}_wm128.log 2>&1 || exit $?
timeout -k 10 200 $B > gpurun_out/${TAG}_default2.log 2>&1 || exit $?
