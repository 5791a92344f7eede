#!/bin/bash
# Round-2 first GPU pass: GPU tests, default bench, 2-rank shard rehearsal (gloo, one GPU),
# rocprofv3 kernel stats of the full bench (L1 + C4 + C5 destriper legs).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02a_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r02a_pytest.log
if [ $rc -ge 2 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/r02a_bench.log 2>&1 || exit $?
COMAP_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 --c5-obs 1 --no-cpu-baseline > gpurun_out/r02a_bench_2rank.log 2>&1 || exit $?
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02a_trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02a_bench_trace.log 2>&1 || exit $?
exit $rc
