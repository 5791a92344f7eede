#!/bin/bash
# HEAD validation after container re-creation: full GPU pytest, smoke, default bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02y_pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02y_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r02y_bench.log 2>&1
