#!/bin/bash
# Round 6: the whole GPU suite, the q-ary fixed-length A/B, deletion bench lines after the guard-band
# scan split (plain scans at n = 8, four-word probes from 128 trellises), and the round's profiles of
# the shipped C2, C4 and C5 kernels.
# usage: OUT=r6c bash scripts/r6_c.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6c}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ab_qary_fixed_n.py > $O/ab_qary_fixed_n.txt 2>&1; rc=$?; tail -3 $O/ab_qary_fixed_n.txt; [ $rc -eq 0 ] || exit $rc
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
run c4 "--workload qary --steps 10 --warmup 3 --no-cpu" || exit 1
WL=deletion TAG=${OUT:-r6c}/del_n8_n02_dense EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=awgn TAG=${OUT:-r6c}/bin_v26_n10 EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=qary TAG=${OUT:-r6c}/qary_q4_n8 EXTRA="" bash scripts/prof_sq.sh || exit 1
exit 0
