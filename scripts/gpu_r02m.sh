#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_c2.py -m gpu -x -v --durations=0 --timeout 400 --timeout-method thread > gpurun_out/r02m_pytest.log 2>&1
