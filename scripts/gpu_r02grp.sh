#!/bin/bash
# B / median / C pipeline groups with the wavelet-matrix median (C2 and a C3 shard), and the
# bench's own 2-rank launch (gloo rehearsal: both ranks share the one GPU).
set -o pipefail
TAG=${1:-r02grp}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_destriper.py -x -v -m gpu --timeout 300 --timeout-method thread -k "compacted or two_ranks" > gpurun_out/${TAG}_compact.log 2>&1 || exit $?
L="--steps 10 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline"
for g in 1 2 3; do
  COMAP_GROUPS=$g timeout -k 10 200 python -u bench.py $L > gpurun_out/${TAG}_c2_g$g.log 2>&1 || exit $?
  COMAP_GROUPS=$g timeout -k 10 200 python -u bench.py $L --shard-of 8 > gpurun_out/${TAG}_s8_g$g.log 2>&1 || exit $?
done
COMAP_GROUPS=2 COMAP_SIDE_PRIO=1 timeout -k 10 200 python -u bench.py $L > gpurun_out/${TAG}_c2_g2p.log 2>&1 || exit $?
COMAP_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 --feeds 6 --no-cpu-baseline --c5-obs 2 --no-e2e > gpurun_out/${TAG}_2rank.log 2>&1 || exit $?
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 1 --warmup 1 --no-cpu-baseline --no-destriper --no-e2e"
timeout -s KILL 180 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum --output-format csv -d gpurun_out/${TAG}_tlb1 -o run -- python3 bench.py $B > gpurun_out/${TAG}_tlb1.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${TAG}_tlb2 -o run -- python3 bench.py $B > gpurun_out/${TAG}_tlb2.log 2>&1 || exit $?
