#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_l1.py tests/test_gpu_destriper.py tests/test_gpu_c2.py tests/test_mapmaking_driver.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02o_pytest.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r02o_bench.log 2>&1 || exit $?
bash scripts/ds_prof_c4.sh r02o > gpurun_out/r02o_c4.log 2>&1
