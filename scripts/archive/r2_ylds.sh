#!/bin/bash
# Re-encoded bits in LDS (variants 24, 25) vs global (17, 20): binary GPU parity for every
# variant, then decode-only bench lines at N = 1024 and N = 4096.
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ylds
cd $R
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ylds/pytest.log 2>&1
rc=$?; echo "pytest decode rc=$rc"; tail -2 gpurun_out/ylds/pytest.log; [ $rc -eq 0 ] || exit $rc
for n in 10 12; do for v in 17 24 20 25; do
  timeout -k 10 300 python bench.py --n $n --variant $v --steps 10 --warmup 3 --no-cpu --no-e2e > gpurun_out/ylds/v${v}_n$n.json 2> gpurun_out/ylds/v${v}_n$n.err
  rc=$?; echo "n=$n v=$v rc=$rc $(python -c "import json; d=json.load(open('gpurun_out/ylds/v${v}_n$n.json')); print('%.2fM cw/s %.2f ms frac %.3f' % (d['value']/1e6, d['roofline']['kernel_ms'], d['roofline']['frac']))")"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/ylds/v${v}_n$n.err; exit $rc; }
done; done
exit 0
