#!/bin/bash
# C4 destriper kernel trace at the full C2 Level-2 size (GPU side).
set -e
export TMPDIR=/tmp
OUT=gpurun_out/ds_c4_${1:-a}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --c5-obs 0 --destriper-iters 200 > $OUT/bench.log 2>&1
find $OUT -name '*kernel_stats.csv' -exec cp {} $OUT/stats.csv \;
