#!/bin/bash
# Round 6: the deletion suite, then C5 / K = 64 bench lines with the 8-lane kernel's rate-1 shortcut
# on and off (interleaved), then the shipped C5 kernel's profile.
# usage: OUT=r6c5 bash scripts/r6_c5.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6c5}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_deletion.py tests/test_gpu_fer.py -x -q --timeout 250 --timeout-method thread > $O/pytest_del.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_del.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for r1 in 1 0; do
    for t in c5 c5k64; do
      case $t in
        c5) A="--workload deletion --steps 10 --warmup 3 --no-cpu";;
        c5k64) A="--workload deletion --del-k 64 --steps 10 --warmup 3 --no-cpu";;
      esac
      timeout -k 10 300 python3 bench.py $A --del-rate1 $r1 > $O/${t}_r1${r1}_$rep.json 2> $O/${t}_r1${r1}_$rep.err; rc=$?
      [ $rc -eq 0 ] || { echo "bench $t rc=$rc"; exit $rc; }
      python3 -c "import json; d=json.load(open('$O/${t}_r1${r1}_$rep.json')); print('$t r1=$r1 rep $rep', round(d['value']/1e6,2), 'M')"
    done
  done
done
WL=deletion TAG=${OUT:-r6c5}/del_n8_n02_dense EXTRA="" bash scripts/prof_sq.sh || exit 1
exit 0
