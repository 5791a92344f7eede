#!/bin/bash
# rocprofv3 kernel stats of the L1 bench (C2) and a C3 shard-of-8
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r02p_c2 -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-destriper --no-e2e --no-cpu-baseline > $R/gpurun_out/r02p_c2.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r02p_s8 -o run -- python3 $R/bench.py --shard-of 8 --steps 5 --warmup 1 --no-destriper --no-e2e --no-cpu-baseline > $R/gpurun_out/r02p_s8.log 2>&1
