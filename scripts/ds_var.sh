#!/bin/bash
# GPU side: C5 destriper leg (tiny L1 leg) for every exp/<name>/libcomap_hip.so, plus optional PMC passes.
mkdir -p gpurun_out
for d in exp/*/; do
  name=$(basename $d)
  COMAP_HIP_LIB=$PWD/exp/$name/libcomap_hip.so timeout -k 10 240 python bench.py --feeds 1 --samples 30000 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/dsvar_$name.log 2>&1 || { echo "variant $name failed rc=$?"; exit 1; }
  echo "variant $name ok"
done
if [ -n "$DS_PMC" ]; then
  export TMPDIR=/tmp
  for name in $DS_PMC; do
    COMAP_HIP_LIB=$PWD/exp/$name/libcomap_hip.so timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/dspmc_$name -o run -- python3 bench.py --feeds 1 --samples 30000 --steps 1 --warmup 0 --no-cpu-baseline --destriper-iters 16 > gpurun_out/dspmc_$name.log 2>&1 || exit 1
    COMAP_HIP_LIB=$PWD/exp/$name/libcomap_hip.so timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/dsfetch_$name -o run -- python3 bench.py --feeds 1 --samples 30000 --steps 1 --warmup 0 --no-cpu-baseline --destriper-iters 16 > gpurun_out/dsfetch_$name.log 2>&1 || exit 1
  done
fi
