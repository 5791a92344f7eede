#!/bin/bash
# Full GPU suite + smoke + default bench at HEAD
set -o pipefail
TAG=${1:-r02p}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
