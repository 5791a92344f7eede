#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02w_c2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-destriper --no-e2e --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r02w_c2.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02w_s8 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --shard-of 8 --steps 5 --warmup 1 --no-destriper --no-e2e --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r02w_s8.log 2>&1
