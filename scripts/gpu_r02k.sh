#!/bin/bash
# median sub-job split A/B (COMAP_MEDIAN_MINSEGS), full C2 and rank 0 of an 8-way C3 split
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_l1.py -m gpu -x -q --timeout 200 --timeout-method thread -k "medfilt or median" > gpurun_out/r02k_pytest.log 2>&1 || exit $?
for m in 0 512 1024 2048; do
  COMAP_MEDIAN_MINSEGS=$m timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02k_c2_m$m.log 2>&1 || exit $?
  COMAP_MEDIAN_MINSEGS=$m timeout -k 10 200 python -u bench.py --shard-of 8 --steps 20 --warmup 3 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02k_s8_m$m.log 2>&1 || exit $?
done
