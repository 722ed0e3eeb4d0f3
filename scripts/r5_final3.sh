#!/bin/bash
# Round 5, final: smoke, the GPU suite, profiles of the C2 and C5 kernels (8-lane deletion layout),
# bench lines for C2 .. C5, C5 K = 64 and the n = 10 / 12 deletion shapes.
# usage: OUT=r5f3 bash scripts/r5_final3.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r5f3}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
WL=awgn TAG=bin_v26_n10 EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=deletion TAG=del_n8_n02_dense EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=deletion TAG=del_n8_n02_k64_dense EXTRA="--del-k 64" bash scripts/prof_sq.sh || exit 1
for t in c2 c3 c4 c5 c5k64 d10 d12; do
  case $t in
    c2) A="--steps 10 --warmup 3";;
    c3) A="--n 12 --steps 5 --warmup 2";;
    c4) A="--workload qary --steps 10 --warmup 3";;
    c5) A="--workload deletion --steps 10 --warmup 3";;
    c5k64) A="--workload deletion --del-k 64 --steps 10 --warmup 3";;
    d10) A="--workload deletion --n 10 --steps 5 --warmup 2 --no-cpu";;
    d12) A="--workload deletion --n 12 --batch 65536 --steps 2 --warmup 1 --no-cpu";;
  esac
  timeout -k 10 400 python3 bench.py $A > $O/$t.json 2> $O/$t.err; rc=$?; echo "bench $t rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('$O/$t.json')); print('  ', d['config']['workload'], round(d['value']/1e6,4), 'M frac', round(d['roofline']['frac'],4))"
done
exit 0
