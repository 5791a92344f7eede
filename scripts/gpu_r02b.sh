#!/bin/bash
# Batched-band destriper: GPU tests of the destriper / mapmaking / noise paths, then the bench.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_destriper.py tests/test_mapmaking_driver.py tests/test_noise_qa.py tests/test_comapdata.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r02b_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r02b_pytest.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r02b_bench.log 2>&1 || exit $?
exit $rc
