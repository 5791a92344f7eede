#!/bin/bash
# median walk: XCD-contiguous chunk order A/B (C2 and rank 0 of an 8-way split)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_l1.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02p_pytest.log 2>&1 || exit $?
for x in 0; do
  COMAP_MEDIAN_XCD=$x timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02p_c2_x$x.log 2>&1 || exit $?
  COMAP_MEDIAN_XCD=$x timeout -k 10 200 python -u bench.py --shard-of 8 --steps 20 --warmup 3 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02p_s8_x$x.log 2>&1 || exit $?
done
