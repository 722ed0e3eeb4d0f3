#!/bin/bash
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_deletion.py tests/test_gpu_leaf.py tests/test_gpu_genie.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_del.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_del.log | tail -5; [ $rc -eq 0 ] || exit $rc
for spec in "n8:" "n8k64:--del-k 64" "n10:--n 10" "n12:--n 12 --batch 262144" "n8ones1:--ones 1"; do
  name=${spec%%:*}; extra=${spec#*:}
  timeout -k 10 400 python bench.py --workload deletion --steps 5 --warmup 2 --no-cpu $extra > gpurun_out/bench_del_$name.json 2> gpurun_out/bench_del_$name.err
  rc=$?; echo "bench del $name rc=$rc $(python -c "import json; d=json.load(open('gpurun_out/bench_del_$name.json')); print('%.2fM cw/s kernel %.2f ms fer %.4f K %d' % (d['value']/1e6, d['roofline']['kernel_ms'], d['fer'], d['config']['K']))")"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/bench_del_$name.err; exit $rc; }
done
exit 0
