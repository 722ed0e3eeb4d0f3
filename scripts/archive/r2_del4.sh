#!/bin/bash
# deletion after the implicit base trellis (n0 >= 3): GPU parity, then n=8 / n=10 bench lines
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_deletion.py tests/test_gpu_leaf.py tests/test_gpu_genie.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_del4.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_del4.log; [ $rc -eq 0 ] || exit $rc
for spec in "n8:" "n10:--n 10 --batch 262144" "n12:--n 12 --batch 32768"; do
  name=${spec%%:*}; extra=${spec#*:}
  timeout -k 10 300 python bench.py --workload deletion --steps 3 --warmup 1 --no-cpu $extra > gpurun_out/bench_del4_$name.json 2> gpurun_out/bench_del4_$name.err
  rc=$?; echo "bench del $name rc=$rc $(python -c "import json; d=json.load(open('gpurun_out/bench_del4_$name.json')); print('%.4fM cw/s kernel %.2f ms' % (d['value']/1e6, d['roofline']['kernel_ms']))")"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/bench_del4_$name.err; exit $rc; }
done
exit 0
