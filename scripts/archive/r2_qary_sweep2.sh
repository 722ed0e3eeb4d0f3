#!/bin/bash
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/qsweep2
cd $R
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -20 gpurun_out/build.log; exit 1; }
for V in "4 0" "4 1" "4 2" "4 3" "8 0" "8 4"; do
  set -- $V
  timeout -k 10 300 python bench.py --workload qary --qregs $1 --qlanes 4 --qvariant $2 --steps 10 --warmup 3 --no-cpu > gpurun_out/qsweep2/s$1_v$2.json 2> gpurun_out/qsweep2/s$1_v$2.err
  rc=$?; echo "S=$1 v=$2 rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/qsweep2/s$1_v$2.json')); print('%.1fM cw/s %.2f ms fer %.4f' % (d['value']/1e6, d['roofline']['kernel_ms'], d['fer']))")"; [ $rc -eq 0 ] || exit $rc
done
for Q in 8 5; do for SG in "0 4" "0 2" "0 1"; do
  set -- $SG
  timeout -k 10 300 python bench.py --workload qary --q $Q --qregs $1 --qlanes $2 --steps 5 --warmup 2 --no-cpu > gpurun_out/qsweep2/q${Q}_s$1_g$2.json 2> gpurun_out/qsweep2/q${Q}_s$1_g$2.err
  rc=$?; echo "q=$Q S=$1 G=$2 rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/qsweep2/q${Q}_s$1_g$2.json')); print('%.1fM cw/s %.2f ms' % (d['value']/1e6, d['roofline']['kernel_ms']))")"; [ $rc -eq 0 ] || exit $rc
done; done
exit 0
