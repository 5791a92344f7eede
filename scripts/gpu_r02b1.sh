#!/bin/bash
# pass B one band per block (k_band_sums1): parity with COMAP_B1=1, then variants
mkdir -p gpurun_out
export TMPDIR=/tmp
COMAP_B1=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_l1.py -m gpu -x -q --timeout 200 --timeout-method thread -k "residues or multi_feed or c1 or averaged or atmosphere or shards or edge_variants or nan_fill" > gpurun_out/r02b1_pytest.log 2>&1 || exit $?
B="--steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline"
COMAP_B1=1 timeout -k 10 200 python -u bench.py $B --check > gpurun_out/r02b1_b18.log 2>&1 || exit $?
for v in b14 b24 b116; do
  COMAP_B1=1 COMAP_HIP_LIB=$PWD/exp/$v/libcomap_hip.so timeout -k 10 200 python -u bench.py $B > gpurun_out/r02b1_$v.log 2>&1 || exit $?
done
