#!/bin/bash
# One parameterised GPU launcher (run on the box through gpurun): each step runs under
# its own time limit, the first failure ends the script (no further GPU step).
#   bash scripts/gpu_run.sh TAG step [step ...]
# steps:  tests[=PYTEST_ARGS]   pytest -m gpu (default: the whole GPU suite)
#         bench[=BENCH_ARGS]    bench.py (default: --steps 5 --warmup 2 --check)
#         prof[=BENCH_ARGS]     rocprofv3 kernel trace + stats of bench.py
#         pmc=COUNTERS[@BENCH_ARGS]  one rocprofv3 --pmc pass
#         smoke                 __graft_entry__.smoke()
#         py=SCRIPT ARGS        python3 SCRIPT ARGS (log gpurun_out/TAG_py<step>.log)
#         pyprof=SCRIPT ARGS    the same under rocprofv3 --kernel-trace --stats (gpurun_out/TAG_pyprof<step>/)
#         dsprof[=ARGS]         rocprofv3 kernel trace + stats of scripts/ds_c5.py (default: 8 obs, 4 bands, 50 it)
#         dspmc=COUNTERS[@ARGS] one rocprofv3 --pmc pass over scripts/ds_c5.py
#         pypmc=COUNTERS@SCRIPT ARGS  one rocprofv3 --pmc pass over python3 SCRIPT ARGS
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
NSTEP=0
for step in "$@"; do
  NSTEP=$((NSTEP + 1))
  name=${step%%=*}; arg=${step#*=}; [ "$arg" = "$step" ] && arg=""
  case $name in
    tests) timeout -k 10 900 python -u -m pytest ${arg:-tests -m gpu} -x -v --timeout 400 --timeout-method thread \
             > gpurun_out/${TAG}_pytest${NSTEP}.log 2>&1 ;;
    bench) timeout -k 10 420 python -u bench.py ${arg:---steps 5 --warmup 2 --check} > gpurun_out/${TAG}_bench.log 2>&1 ;;
    prof)  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run \
             -- python3 bench.py ${arg:---steps 2 --warmup 1 --no-cpu-baseline} > gpurun_out/${TAG}_prof.log 2>&1 ;;
    pmc)   cnt=${arg%%@*}; bargs=${arg#*@}; [ "$bargs" = "$arg" ] && bargs="--steps 1 --warmup 1 --no-cpu-baseline"
           d=gpurun_out/${TAG}_pmc_$(echo $cnt | tr ' ' '_' | cut -c1-40)
           timeout -s KILL 300 rocprofv3 --pmc $cnt --output-format csv -d $d -o run -- python3 bench.py $bargs \
             > $d.log 2>&1 ;;
    dsprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_dstrace${NSTEP} -o run \
             -- python3 scripts/ds_c5.py ${arg:-8 4 50} > gpurun_out/${TAG}_dsprof${NSTEP}.log 2>&1 ;;
    dspmc) cnt=${arg%%@*}; dargs=${arg#*@}; [ "$dargs" = "$arg" ] && dargs="8 4 20"
           d=gpurun_out/${TAG}_dspmc_$(echo $cnt | tr ' ' '_' | cut -c1-40)
           timeout -s KILL 240 rocprofv3 --pmc $cnt --output-format csv -d $d -o run -- python3 scripts/ds_c5.py $dargs \
             > $d.log 2>&1 ;;
    pyprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_pyprof${NSTEP} \
              -o run -- python3 $arg > gpurun_out/${TAG}_pyprof${NSTEP}.log 2>&1 ;;
    pypmc) cnt=${arg%%@*}; sargs=${arg#*@}
           d=gpurun_out/${TAG}_pypmc${NSTEP}
           timeout -s KILL 240 rocprofv3 --pmc $cnt --output-format csv -d $d -o run -- python3 $sargs > $d.log 2>&1 ;;
    py)    timeout -k 10 300 python3 -u $arg > gpurun_out/${TAG}_py${NSTEP}.log 2>&1 ;;
    smoke) timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${TAG}_smoke.log 2>&1 ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
  rc=$?
  echo "step $step rc=$rc" >> gpurun_out/${TAG}_steps.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
