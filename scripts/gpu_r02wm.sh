#!/bin/bash
# wavelet-matrix median walk: median parity (all paths), L1 parity, bench vs bitmap walk
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_l1.py -m gpu -x -v --timeout 200 --timeout-method thread -k "medfilt or median or c1 or averaged or multi_feed or shards" > gpurun_out/r02wm_pytest.log 2>&1 || exit $?
B="--steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline"
timeout -k 10 200 python -u bench.py $B --check > gpurun_out/r02wm_wm.log 2>&1 || exit $?
COMAP_MEDIAN_WALK=bitmap timeout -k 10 200 python -u bench.py $B > gpurun_out/r02wm_bitmap.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py $B --shard-of 8 --steps 20 --warmup 3 > gpurun_out/r02wm_s8.log 2>&1 || exit $?
COMAP_MEDIAN_WALK=bitmap timeout -k 10 200 python -u bench.py $B --shard-of 8 --steps 20 --warmup 3 > gpurun_out/r02wm_s8b.log 2>&1 || exit $?
