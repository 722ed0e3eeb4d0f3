#!/bin/bash
# One GPU session: smoke, parity tests, a bench line, rocprofv3 kernel-trace stats and
# (PMC=1) HBM counter passes.  Every GPU step has its own time limit; the script stops
# at the first crash / timeout.
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
BATCH=${BATCH:-1048576}
# the library is built here (in-tree) before the call; its objects do not travel (.gpurunignore)
if [ -z "${NO_TEST:-}" ]; then
  timeout -k 10 ${T_SMOKE:-300} python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 ${T_TEST:-700} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_EXTRA:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 ${T_BENCH:-400} python bench.py --steps ${STEPS:-10} --warmup 3 --batch $BATCH ${BENCH_EXTRA:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${PROF:-}" ]; then
  cd /tmp
  timeout -k 10 ${T_PROF:-400} rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --batch $BATCH --no-cpu --no-e2e ${BENCH_EXTRA:-} > $R/gpurun_out/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; tail -2 $R/gpurun_out/prof.log
  cd $R
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${PMC:-}" ]; then
  for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=${grp%% *}
    cd /tmp
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc_$tag -o pmc -- python3 $R/scripts/decode_only.py --batch $BATCH --reps 1 ${DECODE_EXTRA:-} > $R/gpurun_out/pmc_$tag.log 2>&1
    rc=$?; echo "pmc $grp rc=$rc"
    cd $R
    [ $rc -eq 0 ] || exit $rc
  done
fi
exit 0
