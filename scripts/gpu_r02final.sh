#!/bin/bash
# Round-2 checkpoint on the GPU box: GPU pytest, smoke, default bench, rocprofv3 stats of the L1 leg.
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
TAG=${1:-r02final}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-destriper --no-e2e > gpurun_out/${TAG}_bench_under_rocprof.log 2>&1 || exit $?
