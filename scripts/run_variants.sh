#!/bin/bash
# GPU side: bench every exp/<name>/libcomap_hip.so (L1 leg only); stops at the first failure.
mkdir -p gpurun_out
for d in exp/*/; do
  name=$(basename $d)
  COMAP_HIP_LIB=$PWD/exp/$name/libcomap_hip.so timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-destriper --check "$@" > gpurun_out/var_$name.log 2>&1 || { echo "variant $name failed rc=$?"; exit 1; }
  echo "variant $name ok"
done
