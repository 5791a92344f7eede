#!/bin/bash
# wide segmented sort A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_l1.py -m gpu -x -q --timeout 200 --timeout-method thread -k "medfilt or median or shards" > gpurun_out/r02x_pytest.log 2>&1 || exit $?
for wd in 0 1; do
  COMAP_SORT_WIDE=$wd timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02x_c2_w$wd.log 2>&1 || exit $?
  COMAP_SORT_WIDE=$wd timeout -k 10 200 python -u bench.py --shard-of 8 --steps 20 --warmup 3 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02x_s8_w$wd.log 2>&1 || exit $?
done
