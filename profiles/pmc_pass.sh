#!/bin/bash
# One rocprofv3 PMC pass over a short bench run (L1 leg only); no trace domains mixed with --pmc.
# usage: bash profiles/pmc_pass.sh TAG "COUNTER COUNTER ..." [bench args]
TAG=$1; CNT=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_$TAG
timeout -s KILL 180 rocprofv3 --pmc $CNT --output-format csv -d gpurun_out/pmc_$TAG -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-destriper "$@" > gpurun_out/pmc_$TAG/bench.log 2>&1
