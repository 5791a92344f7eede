#!/bin/bash
# HEALPix destriper mode through the driver (per-band and batched) on the GPU.
set -o pipefail
TAG=${1:-r02hx}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mapmaking_driver.py tests/test_comapdata.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || exit $?
