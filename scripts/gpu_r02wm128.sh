#!/bin/bash
# WM segment target 128 (default): median parity tests, then the C3 shard and C2 benches
set -o pipefail
TAG=${1:-r02wm128}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_l1.py tests/test_comapdata.py tests/test_gpu_c2.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-destriper --no-e2e --shard-of 8 > gpurun_out/${TAG}_c3.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-destriper --no-e2e > gpurun_out/${TAG}_c2.log 2>&1 || exit $?
