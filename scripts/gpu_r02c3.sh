#!/bin/bash
# C3 strong-scaling rehearsal on one GPU: rank 0's shard of a 2/4/8-way split of the C2 observation.
set -o pipefail
TAG=${1:-r02c3}
mkdir -p gpurun_out
B="--steps 10 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline"
for n in 8 4 2; do
  timeout -k 10 200 python -u bench.py $B --shard-of $n > gpurun_out/${TAG}_shard$n.log 2>&1 || exit $?
done
