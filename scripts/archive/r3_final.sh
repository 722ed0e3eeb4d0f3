#!/bin/bash
# Round 3 closing session: smoke + GPU suite + bench lines of every workload + the deletion
# profiles of the shipped kernels.  Each step time-limited; stops at the first failure.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
line() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$tag.json 2> $O/$tag.err
  local rc=$?; echo "bench $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('$O/$tag.json')); print('  ', d['config']['workload'], round(d['value']/1e6,3), 'M', d['roofline']['kernel'], 'frac', round(d['roofline']['frac'],4), 'e2e', d.get('mc_end_to_end',{}).get('value'))"
}
line c2 --steps 10 --warmup 3
line c3 --n 12 --steps 5 --warmup 2 --no-cpu
line c4 --workload qary --steps 10 --warmup 3 --no-cpu
line c5 --workload deletion --steps 10 --warmup 3
line del_n10 --workload deletion --n 10 --steps 5 --warmup 2 --no-cpu
WL=deletion TAG=del_n8_n02_dense EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=deletion TAG=del_n10_n03_k256_dense EXTRA="--n 10 --batch 1048576" bash scripts/prof_sq.sh
