#!/bin/bash
# One GPU session: parity tests, a bench line, a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; stop at the first crash/timeout.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
BATCH=${BATCH:-1048576}
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 ${T_SMOKE:-300} python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 ${T_TEST:-600} python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in ${VARIANTS:-0 1}; do
  timeout -k 10 ${T_BENCH:-400} python bench.py --steps ${STEPS:-5} --warmup 2 --batch $BATCH --variant $v ${BENCH_EXTRA:-} > gpurun_out/bench_v$v.json 2> gpurun_out/bench_v$v.err
  rc=$?; echo "bench v$v rc=$rc"; cat gpurun_out/bench_v$v.json; tail -3 gpurun_out/bench_v$v.err
  [ $rc -eq 0 ] || exit $rc
done
if [ -n "${PROF:-}" ]; then
  cd /tmp && timeout -k 10 ${T_PROF:-400} rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --batch $BATCH --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; cd $GRAFT_REPO_ROOT
  find gpurun_out/prof -name "*stats*" | head; 
fi
exit 0
