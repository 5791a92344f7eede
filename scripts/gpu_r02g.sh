#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r02g}
timeout -k 10 600 python -u -m pytest tests/test_gpu_destriper.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_pytest.log
exit $rc
