#!/bin/bash
# pass A: default unaligned 16-B loads vs the aligned-chunk kernel with the DPP pair shift (COMAP_A_DPP=1)
set -o pipefail
TAG=${1:-r02dpp}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-destriper --no-e2e"
timeout -k 10 200 $B > gpurun_out/${TAG}_off.log 2>&1 || exit $?
COMAP_A_DPP=1 timeout -k 10 200 $B > gpurun_out/${TAG}_on.log 2>&1 || exit $?
timeout -k 10 200 $B > gpurun_out/${TAG}_off2.log 2>&1 || exit $?
