#!/bin/bash
# Destriper-focused kernel trace (tiny L1 leg, C4-like + C5 legs); GPU side.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/ds_${1:-a}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ds_${1:-a} -o run -- python3 bench.py --feeds 1 --samples 30000 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/ds_${1:-a}/bench.log 2>&1
find gpurun_out/ds_${1:-a} -name '*kernel_stats.csv' -exec cp {} gpurun_out/ds_${1:-a}/stats.csv \;
