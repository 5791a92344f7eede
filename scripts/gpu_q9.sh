mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_q9.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_q9.log 2>&1 || exit 2
COMAP_MEDIAN_PATH=slide timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-destriper > gpurun_out/bench_q9s.log 2>&1 || exit 3
