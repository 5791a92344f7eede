#!/bin/bash
# Address-translation counters per streaming pass (is pass B, which reads 4 KB pieces of ~1000
# rows per tile, paying for translations that the row-streaming passes A and C do not?).
set -o pipefail
TAG=${1:-r02tlb}
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 1 --warmup 1 --no-cpu-baseline --no-destriper --no-e2e"
timeout -s KILL 180 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum --output-format csv -d gpurun_out/${TAG}_p1 -o run -- python3 bench.py $B > gpurun_out/${TAG}_p1.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_p2 -o run -- python3 bench.py $B > gpurun_out/${TAG}_p2.log 2>&1 || exit $?
