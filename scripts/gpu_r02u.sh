#!/bin/bash
# vane split sides; pipeline groups retest with the faster median
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_l1.py tests/test_gpu_c2.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02u_pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02u_c2.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --shard-of 8 --steps 20 --warmup 3 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02u_s8.log 2>&1 || exit $?
COMAP_GROUPS=2 timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02u_c2_g2.log 2>&1 || exit $?
COMAP_GROUPS=2 COMAP_SIDE_PRIO=1 timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02u_c2_g2p.log 2>&1 || exit $?
COMAP_GROUPS=2 timeout -k 10 200 python -u bench.py --shard-of 8 --steps 20 --warmup 3 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02u_s8_g2.log 2>&1 || exit $?
