#!/bin/bash
# L1 median overlap A/B: unit groups x median side-stream priority (bench L1 leg only).
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "1 0" "2 0" "2 1" "4 0" "4 1"; do
  set -- $cfg
  COMAP_GROUPS=$1 COMAP_SIDE_PRIO=$2 timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02h_g$1_p$2.log 2>&1 || exit $?
done
