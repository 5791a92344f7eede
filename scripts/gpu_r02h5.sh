#!/bin/bash
# HDF5 file layer on the GPU box: the Runner-from-HDF5 parity test, the full GPU suite, file -> HBM staging rate.
set -o pipefail
TAG=${1:-r02h5}
mkdir -p gpurun_out
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 300 python -u -m pytest tests/test_gpu_hdf5.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_hdf5.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/h5_upload.py 2 180000 > gpurun_out/${TAG}_upload.log 2>&1 || exit $?
