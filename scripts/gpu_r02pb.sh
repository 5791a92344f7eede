#!/bin/bash
# median proxy bits 24 vs 32, two-group B/median/C pipeline; median parity
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_l1.py -m gpu -x -q --timeout 200 --timeout-method thread -k "medfilt or median or c1" > gpurun_out/r02pb_pytest.log 2>&1 || exit $?
B="--steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline"
timeout -k 10 200 python -u bench.py $B > gpurun_out/r02pb_24.log 2>&1 || exit $?
COMAP_MEDIAN_PBITS=32 timeout -k 10 200 python -u bench.py $B > gpurun_out/r02pb_32.log 2>&1 || exit $?
COMAP_GROUPS=2 timeout -k 10 200 python -u bench.py $B --check > gpurun_out/r02pb_g2.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py $B --shard-of 8 --steps 20 --warmup 3 > gpurun_out/r02pb_s8.log 2>&1 || exit $?
COMAP_MEDIAN_PBITS=32 timeout -k 10 200 python -u bench.py $B --shard-of 8 --steps 20 --warmup 3 > gpurun_out/r02pb_s832.log 2>&1 || exit $?
