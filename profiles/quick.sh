#!/bin/bash
# Quick GPU iteration: pytest -m gpu then a short bench (no CPU baseline).
# usage: bash profiles/quick.sh TAG [extra bench args]
TAG=${1:-q}; shift || true
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_${TAG}.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --check "$@" > gpurun_out/bench_${TAG}.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench_${TAG}.log
exit $rc
