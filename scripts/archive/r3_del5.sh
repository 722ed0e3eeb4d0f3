#!/bin/bash
# round 3: deletion through the table-driven layout -- bench lines (C5 K=3, K=64, n = 10, 11, 12)
# and the C5 / n = 10 profiles (trace, HBM, SQ mix)
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 200 python3 bench.py --workload deletion "$@" --steps 5 --warmup 2 --no-e2e > gpurun_out/$tag.json 2> gpurun_out/$tag.err
  local rc=$?; echo "bench $tag rc=$rc"; cat gpurun_out/$tag.json; [ $rc -eq 0 ] || exit $rc
}
run del5_c5
run del5_c5_k64 --del-k 64 --no-cpu
run del5_n10 --n 10 --batch 1048576
run del5_n11 --n 11 --batch 262144 --no-cpu
run del5_n12 --n 12 --batch 8192 --no-cpu
WL=deletion TAG=del_n8_dense EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=deletion TAG=del_n10_dense EXTRA="--n 10 --batch 1048576" bash scripts/prof_sq.sh
