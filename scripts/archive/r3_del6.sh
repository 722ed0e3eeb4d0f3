#!/bin/bash
# round 3: deletion tests + bench lines after the unrolled row packing
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_deletion.py tests/test_gpu_genie.py tests/test_gpu_leaf.py -x -q --timeout 120 --timeout-method thread > gpurun_out/del6_test.log 2>&1
rc=$?; tail -3 gpurun_out/del6_test.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 200 python3 bench.py --workload deletion "$@" --steps 5 --warmup 2 --no-e2e --no-cpu > gpurun_out/$tag.json 2> gpurun_out/$tag.err
  local rc=$?; echo "bench $tag rc=$rc"; python3 -c "import json,sys; d=json.load(open('gpurun_out/$tag.json')); print(d['config']['workload'], round(d['value']/1e6,2), 'M', d['roofline']['kernel'], round(d['roofline']['kernel_ms'],3))"; [ $rc -eq 0 ] || exit $rc
}
run del6_c5
run del6_c5_k64 --del-k 64
run del6_n10 --n 10 --batch 1048576
run del6_n11 --n 11 --batch 262144
timeout -k 10 300 python -u scripts/del_table.py > gpurun_out/del6_time.log 2>&1; rc=$?; cat gpurun_out/del6_time.log; exit $rc
