#!/bin/bash
# Round 6 final check: smoke, the whole GPU suite, and the bench lines of every BASELINE config the
# driver's default run does not cover (C3 per GPU, C4, C5, C5 K = 64, deletion n = 10 .. 14), plus C2
# with its CPU baseline.
# usage: OUT=r6d bash scripts/r6_d.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6d}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, args
  timeout -k 10 400 python3 bench.py $2 > $O/$1.json 2> $O/$1.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench $1 rc=$rc"; tail -3 $O/$1.err; return $rc; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); e=d.get('mc_end_to_end',{}); print('$1', round(d['value']/1e6,4), 'M  frac', round(d['roofline']['frac'],4), ' e2e', round(e.get('value',0)/1e6,2))"
}
run c2 "--steps 10 --warmup 3" || exit 1
run c3 "--n 12 --steps 5 --warmup 2" || exit 1
run c4 "--workload qary --steps 10 --warmup 3" || exit 1
run c5 "--workload deletion --steps 10 --warmup 3" || exit 1
run c5k64 "--workload deletion --del-k 64 --steps 10 --warmup 3 --no-cpu" || exit 1
run d9 "--workload deletion --n 9 --steps 5 --warmup 2 --no-cpu" || exit 1
run d10 "--workload deletion --n 10 --steps 5 --warmup 2 --no-cpu" || exit 1
run d11 "--workload deletion --n 11 --batch 262144 --steps 5 --warmup 2 --no-cpu" || exit 1
run d12 "--workload deletion --n 12 --batch 32768 --steps 2 --warmup 1 --no-cpu" || exit 1
run n13 "--n 13 --batch 262144 --steps 5 --warmup 2 --no-cpu" || exit 1
run scl "--workload scl --no-cpu" || exit 1
exit 0
