#!/bin/bash
# LDS-privatised scatter bin vs pixel-major gather at C5 (8 obs, 1 and 4 bands), with kernel stats
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_destriper.py -m gpu -x -q --timeout 200 --timeout-method thread -k "lds or offset_lengths or batched_bands" > gpurun_out/r02t_pytest.log 2>&1 || exit $?
for nb in 1 4; do
  timeout -k 10 200 python -u scripts/ds_c5.py 8 $nb 50 > gpurun_out/r02t_gather_b$nb.log 2>&1 || exit $?
  for t in 128 256 512 1024; do
    COMAP_DS_BIN=lds COMAP_DS_TILE=$t timeout -k 10 200 python -u scripts/ds_c5.py 8 $nb 50 > gpurun_out/r02t_lds${t}_b$nb.log 2>&1 || exit $?
  done
done
cd /tmp && COMAP_DS_BIN=lds COMAP_DS_TILE=256 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02t_trace -o run -- python3 $GRAFT_REPO_ROOT/scripts/ds_c5.py 8 4 30 > $GRAFT_REPO_ROOT/gpurun_out/r02t_trace.log 2>&1
