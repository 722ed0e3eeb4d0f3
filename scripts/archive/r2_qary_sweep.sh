#!/bin/bash
# q-ary geometry sweep (S register positions x G lanes), q = 4 N = 256 on the C4 code.
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/qsweep
cd $R
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_qary.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_qary.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_qary.log; [ $rc -eq 0 ] || exit $rc
for SG in "8 4" "4 4" "8 2" "4 2" "8 1" "4 1"; do
  set -- $SG
  timeout -k 10 300 python bench.py --workload qary --qregs $1 --qlanes $2 --steps 10 --warmup 3 --no-cpu > gpurun_out/qsweep/q4_s$1_g$2.json 2> gpurun_out/qsweep/q4_s$1_g$2.err
  rc=$?; echo "S=$1 G=$2 rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/qsweep/q4_s$1_g$2.json')); print('%.1fM cw/s %.2f ms' % (d['value']/1e6, d['roofline']['kernel_ms']))")"; [ $rc -eq 0 ] || exit $rc
done
for Q in 3 8; do for SG in "0 4" "2 4" "0 2"; do
  set -- $SG
  timeout -k 10 300 python bench.py --workload qary --q $Q --qregs $1 --qlanes $2 --steps 5 --warmup 2 --no-cpu > gpurun_out/qsweep/q${Q}_s$1_g$2.json 2> gpurun_out/qsweep/q${Q}_s$1_g$2.err
  rc=$?; echo "q=$Q S=$1 G=$2 rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/qsweep/q${Q}_s$1_g$2.json')); print('%.1fM cw/s %.2f ms' % (d['value']/1e6, d['roofline']['kernel_ms']))")"; [ $rc -eq 0 ] || exit $rc
done; done
exit 0
