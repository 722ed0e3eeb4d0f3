#!/bin/bash
# Round 4 closing session: smoke + the whole GPU suite + the bench lines of every BASELINE workload
# + the q-ary profile of the shipped kernel.  Each step time-limited; stops at the first failure.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final4
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
line() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err
  local rc=$?; echo "bench $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('$O/$tag.json')); print('  ', d['config']['workload'], round(d['value']/1e6,3), 'M', d['roofline']['kernel'], 'frac', round(d['roofline']['frac'],4), 'e2e', d.get('mc_end_to_end',{}).get('value'), 'cpu', d.get('cpu_baseline',{}).get('value'))"
}
line c2 --steps 10 --warmup 3
line c4 --workload qary --steps 10 --warmup 3
line c5 --workload deletion --steps 10 --warmup 3
line c3 --n 12 --steps 5 --warmup 2 --no-cpu
WL=qary TAG=qary_q4_n8 EXTRA="" bash scripts/prof_sq.sh
