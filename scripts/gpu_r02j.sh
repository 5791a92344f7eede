#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r02j}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u bench.py --shard-of 8 --steps 20 --warmup 3 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/${T}_shard8.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || exit $?
