#!/bin/bash
# aligned pass A (k_moments_al): parity of every scan residue, then old vs new
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_l1.py -m gpu -x -q --timeout 200 --timeout-method thread -k "residues or multi_feed or c1 or averaged or atmosphere or shards or edge_variants" > gpurun_out/r02z_pytest.log 2>&1 || exit $?
B="--steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline"
COMAP_A_DPP=0 timeout -k 10 200 python -u bench.py $B > gpurun_out/r02z_old.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py $B > gpurun_out/r02z_vA.log 2>&1 || exit $?
for g in 2 4; do COMAP_GROUPS=$g timeout -k 10 200 python -u bench.py $B > gpurun_out/r02z_g$g.log 2>&1 || exit $?; done
