#!/bin/bash
# row-stride sensitivity of the streaming passes: the C2 cube at T = 180000 vs nearby sample counts
set -o pipefail
TAG=${1:-r02tp}
mkdir -p gpurun_out
export TMPDIR=/tmp
for T in 180000 180224 180032 181248 180000; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-destriper --no-e2e --samples $T > gpurun_out/${TAG}_T$T.log 2>&1 || exit $?
done
