#!/bin/bash
# Per-rank cost of C3 at N = 2, 4, 8: rank 0's shard reduced alone on one GPU.
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 2 4 8; do
  timeout -k 10 200 python -u bench.py --shard-of $n --steps 20 --warmup 3 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02i_shard$n.log 2>&1 || exit $?
done
