#!/bin/bash
# walk: chunks per workgroup (COMAP_MEDIAN_S) A/B, C2 and rank 0 of an 8-way split
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in 1 2 4 16; do
  COMAP_MEDIAN_S=$s timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02r_c2_s$s.log 2>&1 || exit $?
  COMAP_MEDIAN_S=$s timeout -k 10 200 python -u bench.py --shard-of 8 --steps 20 --warmup 3 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02r_s8_s$s.log 2>&1 || exit $?
done
