#!/bin/bash
# GPU validation run used with gpurun: pytest -m gpu, then a short bench.
# A test failure (rc 1) still lets the bench run; any fault/abort/timeout
# (rc >= 2) stops the script before anything else touches the GPU.
# usage: bash profiles/gpu_check.sh TAG
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_${TAG}.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --check > gpurun_out/bench_${TAG}.log 2>&1
rc2=$?
echo "bench rc=$rc2" >> gpurun_out/bench_${TAG}.log
if [ $rc2 -ne 0 ]; then exit $rc2; fi
exit $rc
