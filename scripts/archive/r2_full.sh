#!/bin/bash
# Full GPU check: smoke, the whole -m gpu suite, one bench line per workload (+ rocprofv3 kernel
# trace per workload when PROF=1).  Every GPU step has its own limit; stop at the first failure.
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for spec in ${SPECS:-"awgn:" "qary:" "deletion:" "awgn12:--n 12"}; do
  name=${spec%%:*}; extra=${spec#*:}
  wl=${name%12}
  timeout -k 10 400 python bench.py --workload $wl --steps ${STEPS:-10} --warmup 3 $extra ${BENCH_EXTRA:-} > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.err
  rc=$?; echo "bench $name rc=$rc $(python -c "import json; d=json.load(open('gpurun_out/bench_$name.json')); print('%.1fM cw/s kernel %.2f ms frac %.3f cpu %s' % (d['value']/1e6, d['roofline']['kernel_ms'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value')))")"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/bench_$name.err; exit $rc; }
  if [ -n "${PROF:-}" ]; then
    cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$name/trace -o run -- python3 $R/bench.py --workload $wl --steps 3 --warmup 1 --no-cpu --no-e2e $extra > $R/gpurun_out/prof_$name.log 2>&1
    rc=$?; echo "prof $name rc=$rc"; cd $R
    [ $rc -eq 0 ] || exit $rc
  fi
done
exit 0
