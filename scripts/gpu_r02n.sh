#!/bin/bash
set -e
bash profiles/profile.sh r02 --steps 2 --warmup 1 --no-cpu-baseline --no-destriper --no-e2e > gpurun_out/r02n_l1.log 2>&1
bash profiles/profile_ds.sh r02_c5 8 4 30 > gpurun_out/r02n_ds.log 2>&1
bash scripts/ds_prof_c4.sh r02n > gpurun_out/r02n_c4.log 2>&1
