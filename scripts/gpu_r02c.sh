#!/bin/bash
# Full GPU pass: pytest -m gpu, default bench, kernel stats of the bench and of the C5
# destriper (1 and 4 bands), FETCH/WRITE PMC of the C5 destriper (separate passes).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02c_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r02c_pytest.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/r02c_bench.log 2>&1 || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02c_trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02c_bench_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02c_ds1 -o run -- python3 scripts/ds_c5.py 8 1 50 > gpurun_out/r02c_ds1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02c_ds4 -o run -- python3 scripts/ds_c5.py 8 4 50 > gpurun_out/r02c_ds4.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r02c_ds4_fetch -o run -- python3 scripts/ds_c5.py 8 4 20 > gpurun_out/r02c_ds4_fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r02c_ds4_write -o run -- python3 scripts/ds_c5.py 8 4 20 > gpurun_out/r02c_ds4_write.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r02c_ds1_fetch -o run -- python3 scripts/ds_c5.py 8 1 20 > gpurun_out/r02c_ds1_fetch.log 2>&1 || exit $?
exit $rc
