#!/bin/bash
# q-ary symbols in LDS: q-ary GPU parity, C4 bench lines with and without, then the full check.
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/qlds
cd $R
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_qary.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/qlds/pytest.log 2>&1
rc=$?; echo "pytest qary rc=$rc"; tail -2 gpurun_out/qlds/pytest.log; [ $rc -eq 0 ] || exit $rc
for l in 1 0; do
  timeout -k 10 300 python bench.py --workload qary --qlds $l --steps 10 --warmup 3 --no-cpu --no-e2e > gpurun_out/qlds/l$l.json 2> gpurun_out/qlds/l$l.err
  rc=$?; echo "qlds=$l rc=$rc $(python -c "import json; d=json.load(open('gpurun_out/qlds/l$l.json')); print('%.2fM cw/s %.2f ms frac %.3f' % (d['value']/1e6, d['roofline']['kernel_ms'], d['roofline']['frac']))")"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/qlds/l$l.err; exit $rc; }
done
bash scripts/r2_full.sh
