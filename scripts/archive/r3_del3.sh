#!/bin/bash
# round 3: n0 = 3 deletion through the segment-state table -- bench lines at n = 10, 11, 12 and
# the n = 10 profile (trace, HBM, SQ mix)
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for nb in "10 262144" "11 65536" "12 8192"; do
  set -- $nb
  timeout -k 10 200 python3 bench.py --workload deletion --n $1 --batch $2 --steps 3 --warmup 1 --no-cpu --no-e2e > gpurun_out/del3_n$1.json 2> gpurun_out/del3_n$1.err
  rc=$?; echo "bench n=$1 rc=$rc"; cat gpurun_out/del3_n$1.json; [ $rc -eq 0 ] || exit $rc
done
WL=deletion TAG=del_n10_n03_tab EXTRA="--n 10 --batch 262144" bash scripts/prof_sq.sh
