#!/bin/bash
# Secondary workloads (BASELINE configs[2..4]) + the headline, one bench line each, and a
# kernel-trace profile per workload.  Every GPU step has its own limit; stop on the first failure.
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
for spec in ${SPECS:-"awgn:" "deletion:" "qary:" "awgn12:--n 12"}; do
  name=${spec%%:*}; extra=${spec#*:}
  wl=${name%12}
  timeout -k 10 ${T_BENCH:-400} python bench.py --workload $wl --steps ${STEPS:-5} --warmup 2 $extra ${BENCH_EXTRA:-} > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.err
  rc=$?; echo "bench $name rc=$rc"; cat gpurun_out/bench_$name.json; tail -2 gpurun_out/bench_$name.err
  [ $rc -eq 0 ] || exit $rc
  if [ -n "${PROF:-}" ]; then
    cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$name -o run -- python3 $R/bench.py --workload $wl --steps 3 --warmup 1 --no-cpu $extra > $R/gpurun_out/prof_$name.log 2>&1
    rc=$?; echo "prof $name rc=$rc"; cd $R
    [ $rc -eq 0 ] || exit $rc
  fi
done
exit 0
