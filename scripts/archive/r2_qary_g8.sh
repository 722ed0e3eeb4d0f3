#!/bin/bash
# q-ary G = 8 / 16 geometries (one / two stored stage levels fewer): q-ary GPU parity, then
# a bench line per geometry at C4 (q = 4, N = 256, the reference C4 frozen set).
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/qg8
cd $R
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_qary.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/qg8/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/qg8/pytest.log; [ $rc -eq 0 ] || exit $rc
for V in "4 4" "4 8" "8 8" "2 8" "4 16" "2 16"; do
  set -- $V
  timeout -k 10 300 python bench.py --workload qary --qregs $1 --qlanes $2 --steps 10 --warmup 3 --no-cpu --no-e2e > gpurun_out/qg8/s$1_g$2.json 2> gpurun_out/qg8/s$1_g$2.err
  rc=$?; echo "S=$1 G=$2 rc=$rc $(python -c "import json,sys; d=json.load(open('gpurun_out/qg8/s$1_g$2.json')); print('%.1fM cw/s %.2f ms frac %.3f' % (d['value']/1e6, d['roofline']['kernel_ms'], d['roofline']['frac']))")"; [ $rc -eq 0 ] || exit $rc
done
exit 0
