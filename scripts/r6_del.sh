#!/bin/bash
# Round 6: the deletion suite, then deletion bench lines (C5, K = 64, n = 10 / 11 / 12) after the
# guard-band scan change, and the shipped C5 kernel's profile.
# usage: OUT=r6del bash scripts/r6_del.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6del}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_deletion.py tests/test_gpu_genie.py tests/test_gpu_fer.py tests/test_gpu_mc.py -x -q --timeout 250 --timeout-method thread > $O/pytest_del.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_del.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, args
  timeout -k 10 400 python3 bench.py $2 > $O/$1.json 2> $O/$1.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench $1 rc=$rc"; tail -3 $O/$1.err; return $rc; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('$1', round(d['value']/1e6,4), 'M  frac', round(d['roofline']['frac'],4))"
}
for rep in 1 2; do
  run c5_$rep "--workload deletion --steps 10 --warmup 3 --no-cpu" || exit 1
  run c5k64_$rep "--workload deletion --del-k 64 --steps 10 --warmup 3 --no-cpu" || exit 1
  run d10_$rep "--workload deletion --n 10 --steps 5 --warmup 2 --no-cpu" || exit 1
done
run d11 "--workload deletion --n 11 --batch 262144 --steps 5 --warmup 2 --no-cpu" || exit 1
run d12 "--workload deletion --n 12 --batch 32768 --steps 2 --warmup 1 --no-cpu" || exit 1
WL=deletion TAG=${OUT:-r6del}/del_n8_n02_dense EXTRA="" bash scripts/prof_sq.sh || exit 1
exit 0
