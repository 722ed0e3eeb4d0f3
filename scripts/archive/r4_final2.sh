#!/bin/bash
# Round 4, last check of the shipped tree: smoke, the whole GPU suite, the C2 / C4 bench lines.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final5
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_tr.py > $O/ab_tr.txt 2>&1; rc=$?; echo "ab rc=$rc"; tail -3 $O/ab_tr.txt; [ $rc -eq 0 ] || exit $rc
for t in c2 c4; do
  if [ $t = c2 ]; then A="--steps 10 --warmup 3"; else A="--workload qary --steps 10 --warmup 3"; fi
  timeout -k 10 400 python3 bench.py $A > $O/$t.json 2> $O/$t.err; rc=$?; echo "bench $t rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('$O/$t.json')); print('  ', d['config']['workload'], round(d['value']/1e6,3), 'M frac', round(d['roofline']['frac'],4), 'e2e', d.get('mc_end_to_end',{}).get('value'))"
done
