#!/bin/bash
# 4-ary wavelet-matrix median walk: median + L1 parity, bench wm4 vs wm2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_l1.py -m gpu -x -q --timeout 200 --timeout-method thread -k "medfilt or median or c1 or multi_feed or shards or residues" > gpurun_out/r02wq_pytest.log 2>&1 || exit $?
B="--steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline"
timeout -k 10 200 python -u bench.py $B --check > gpurun_out/r02wq_wm4.log 2>&1 || exit $?
COMAP_MEDIAN_WALK=wm2 timeout -k 10 200 python -u bench.py $B > gpurun_out/r02wq_wm2.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py $B --shard-of 8 --steps 20 --warmup 3 > gpurun_out/r02wq_s8.log 2>&1 || exit $?
COMAP_MEDIAN_WALK=wm2 timeout -k 10 200 python -u bench.py $B --shard-of 8 --steps 20 --warmup 3 > gpurun_out/r02wq_s8w2.log 2>&1 || exit $?
