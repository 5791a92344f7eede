#!/bin/bash
# Kernel trace of rank 0's C3 shard (8-way split of the C2 observation) on one GPU.
set -o pipefail
TAG=${1:-r02s8}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-destriper --no-e2e --shard-of 8 > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
