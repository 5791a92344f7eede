#!/bin/bash
# 2-rank rehearsal of bench.py's N > 1 path on ONE GPU (gloo backend, both ranks on cuda:0):
# the C3 shard, the C5 legs and the configs[4] field with its work-balanced split and
# per-rank report.  Usage: bash scripts/rehearse_2rank_bench.sh TAG
TAG=${1:-r2}
mkdir -p gpurun_out
COMAP_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 --feeds 6 \
  --no-cpu-baseline --c5-obs 2 --no-e2e --no-chain > gpurun_out/${TAG}_bench_2rank_gloo.log 2>&1
