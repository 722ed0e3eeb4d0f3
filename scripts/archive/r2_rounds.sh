#!/bin/bash
# Whole-round persistent grids: binary / q-ary parity, then bench lines.
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/rounds
cd $R
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_qary.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rounds/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/rounds/pytest.log; [ $rc -eq 0 ] || exit $rc
for spec in "awgn:" "awgn12:--n 12" "qary:" "awgn_b18:--batch 262144"; do
  name=${spec%%:*}; extra=${spec#*:}; wl=${name%%12}; wl=${wl%%_b18}
  timeout -k 10 300 python bench.py --workload $wl $extra --steps 10 --warmup 3 --no-cpu --no-e2e > gpurun_out/rounds/$name.json 2> gpurun_out/rounds/$name.err
  rc=$?; echo "$name rc=$rc $(python -c "import json; d=json.load(open('gpurun_out/rounds/$name.json')); print('%.2fM cw/s %.2f ms frac %.3f' % (d['value']/1e6, d['roofline']['kernel_ms'], d['roofline']['frac']))")"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/rounds/$name.err; exit $rc; }
done
exit 0
