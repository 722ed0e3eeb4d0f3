#!/bin/bash
# n0 = 2 collapse over gathered paths: deletion GPU parity, the configs[4] bench line, VALU count.
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/del5
cd $R
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_deletion.py tests/test_gpu_leaf.py tests/test_gpu_genie.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/del5/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/del5/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload deletion --steps 10 --warmup 3 --no-cpu > gpurun_out/del5/bench_n8.json 2> gpurun_out/del5/bench_n8.err
rc=$?; echo "bench n8 rc=$rc $(python -c "import json; d=json.load(open('gpurun_out/del5/bench_n8.json')); print('%.2fM cw/s %.2f ms fer %.4f' % (d['value']/1e6, d['roofline']['kernel_ms'], d['fer']))")"; [ $rc -eq 0 ] || exit $rc
TAG=del5_n8 ARGS="--workload deletion" NO_TRACE=1 PASSES="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH" bash scripts/prof_passes.sh || exit 1
exit 0
