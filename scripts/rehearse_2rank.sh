mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_destriper.py -x -v -m gpu --timeout 200 --timeout-method thread -k two_ranks > gpurun_out/pytest_2rank.log 2>&1 || exit $?
COMAP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 --feeds 6 --no-cpu-baseline --c5-obs 2 > gpurun_out/bench_2rank.log 2>&1
