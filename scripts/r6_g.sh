#!/bin/bash
# Round 6 final profiles (kernel trace + HBM + SQ passes) of the shipped kernels with counter tiles:
# C2 (variant 26), C3's N = 4096 (variant 30), C4, C5 and C5 K = 64; and their bench lines.
# usage: OUT=r6g bash scripts/r6_g.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6g}
mkdir -p $O
run() {  # tag, args
  timeout -k 10 400 python3 bench.py $2 > $O/$1.json 2> $O/$1.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench $1 rc=$rc"; tail -3 $O/$1.err; return $rc; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); e=d.get('mc_end_to_end',{}); print('$1', round(d['value']/1e6,4), 'M  frac', round(d['roofline']['frac'],4), ' e2e', round(e.get('value',0)/1e6,2))"
}
WL=awgn TAG=${OUT:-r6g}/bin_v26_n10 EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=awgn TAG=${OUT:-r6g}/bin_v30_n12 EXTRA="--n 12" bash scripts/prof_sq.sh || exit 1
WL=qary TAG=${OUT:-r6g}/qary_q4_n8 EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=deletion TAG=${OUT:-r6g}/del_n8_n02_dense EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=deletion TAG=${OUT:-r6g}/del_n8_n02_k64_dense EXTRA="--del-k 64" bash scripts/prof_sq.sh || exit 1
run c2 "--steps 10 --warmup 3" || exit 1
run c3 "--n 12 --steps 5 --warmup 2" || exit 1
run c4 "--workload qary --steps 10 --warmup 3" || exit 1
run c5 "--workload deletion --steps 10 --warmup 3" || exit 1
run c5k64 "--workload deletion --del-k 64 --steps 10 --warmup 3 --no-cpu" || exit 1
run d11 "--workload deletion --n 11 --batch 262144 --steps 5 --warmup 2 --no-cpu" || exit 1
run n13 "--n 13 --batch 262144 --steps 5 --warmup 2 --no-cpu" || exit 1
exit 0
