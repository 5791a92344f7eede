#!/bin/bash
# Pass B layouts (COMAP_B1), pipeline groups, compacted multi-rank destriper, 2-rank self-launch, TLB counters.
set -o pipefail
TAG=${1:-r02bv}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_destriper.py tests/test_gpu_l1.py -x -v -m gpu --timeout 300 --timeout-method thread -k "compacted or two_ranks or pass_b_layouts" > gpurun_out/${TAG}_tests.log 2>&1 || exit $?
L="--steps 10 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline"
for v in 0 1 2 4 8; do
  COMAP_B1=$v timeout -k 10 200 python -u bench.py $L > gpurun_out/${TAG}_b1_$v.log 2>&1 || exit $?
done
for g in 2 3; do
  COMAP_GROUPS=$g timeout -k 10 200 python -u bench.py $L > gpurun_out/${TAG}_c2_g$g.log 2>&1 || exit $?
done
B="--steps 1 --warmup 1 --no-cpu-baseline --no-destriper --no-e2e"
timeout -s KILL 180 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum --output-format csv -d gpurun_out/${TAG}_tlb1 -o run -- python3 bench.py $B > gpurun_out/${TAG}_tlb1.log 2>&1 || exit $?
COMAP_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 --feeds 6 --no-cpu-baseline --c5-obs 2 --no-e2e > gpurun_out/${TAG}_2rank.log 2>&1 || exit $?
