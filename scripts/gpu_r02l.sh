#!/bin/bash
# median: 32-bit proxy sort vs u64 sort, walk chunk 128/256/512; C2 and rank 0 of an 8-way C3 split
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_l1.py tests/test_comapdata.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02l_pytest.log 2>&1 || exit $?
for v in "1 128" "1 64"; do
  set -- $v
  COMAP_MEDIAN_KEY32=$1 COMAP_MEDIAN_L=$2 timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02l_c2_k$1_l$2.log 2>&1 || exit $?
  COMAP_MEDIAN_KEY32=$1 COMAP_MEDIAN_L=$2 timeout -k 10 200 python -u bench.py --shard-of 8 --steps 20 --warmup 3 --no-destriper --no-e2e --no-cpu-baseline > gpurun_out/r02l_s8_k$1_l$2.log 2>&1 || exit $?
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02l_trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-destriper --no-e2e --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r02l_trace.log 2>&1
