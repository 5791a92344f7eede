#!/bin/bash
# Round-2 evidence at HEAD: GPU suite, smoke, default bench (as the driver runs it), rocprofv3 stats +
# FETCH/WRITE traffic of the L1 bench and of the C5 destriper (4 bands).
set -o pipefail
TAG=${1:-r02m}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
bash profiles/profile.sh ${TAG} --steps 3 --warmup 1 --no-cpu-baseline --no-destriper --no-e2e || exit $?
bash profiles/profile_ds.sh ${TAG}_c5 8 4 30 || exit $?
