#!/bin/bash
# SQ counters of the L1 bench kernels (median walk focus), one pass
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_r02s
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc_r02s -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-destriper --no-e2e > gpurun_out/pmc_r02s/bench.log 2>&1
