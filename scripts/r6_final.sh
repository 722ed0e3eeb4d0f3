#!/bin/bash
# Round 6 closing check: smoke, the whole GPU suite, and the bench lines (C2 default, C5, n0 = 4).
# usage: OUT=r6final bash scripts/r6_final.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6final}
mkdir -p $O
cd $R
run() {  # tag, args
  timeout -k 10 400 python3 bench.py $2 > $O/$1.json 2> $O/$1.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench $1 rc=$rc"; tail -3 $O/$1.err; return $rc; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('$1', round(d['value']/1e3,2), 'k cw/s  kernel', d['roofline'].get('kernel'), 'frac', round(d['roofline']['frac'],4))"
}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1200 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run c2 "--steps 10 --warmup 3" || exit 1
run c5 "--workload deletion --steps 10 --warmup 3" || exit 1
run d12 "--workload deletion --n 12 --batch 32768 --steps 3 --warmup 1 --no-cpu" || exit 1
run d13 "--workload deletion --n 13 --batch 16384 --steps 3 --warmup 1 --no-cpu" || exit 1
run d14 "--workload deletion --n 14 --batch 8192 --steps 3 --warmup 1 --no-cpu" || exit 1
run d12_lane "--workload deletion --n 12 --batch 8192 --steps 2 --warmup 1 --no-cpu --del-wave 0" || exit 1
run d14_lane "--workload deletion --n 14 --batch 4096 --steps 2 --warmup 1 --no-cpu --del-wave 0" || exit 1
exit 0
