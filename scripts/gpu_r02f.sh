#!/bin/bash
# Destriper offset order A/B: parity tests, C5 kernel stats with the spatial order (default) and time order.
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r02f}
timeout -k 10 600 python -u -m pytest tests/test_gpu_destriper.py tests/test_mapmaking_driver.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_ds1 -o run -- python3 scripts/ds_c5.py 8 1 50 > gpurun_out/${T}_ds1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_ds4 -o run -- python3 scripts/ds_c5.py 8 4 50 > gpurun_out/${T}_ds4.log 2>&1 || exit $?
COMAP_DS_ORDER=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_ds4t -o run -- python3 scripts/ds_c5.py 8 4 50 > gpurun_out/${T}_ds4t.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/${T}_bench.log 2>&1 || exit $?
