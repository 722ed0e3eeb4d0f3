#!/bin/bash
# Round 5: the dense-slot trellises (trellis_dense.h) on the n0 >= 3 lane kernels -- the GPU suite,
# then the deletion bench at main_deletion.py's n0 = n // 3 for n = 12, 13, 14 (n0 = 4).
# usage: OUT=r5n04 bash scripts/r5_n04.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r5n04}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for n in 12 13 14; do
  case $n in 12) B=65536;; 13) B=32768;; 14) B=16384;; esac
  timeout -k 10 300 python3 bench.py --workload deletion --n $n --batch $B --steps 2 --warmup 1 --no-cpu --no-e2e > $O/del_n$n.json 2> $O/del_n$n.err; rc=$?
  echo "bench n$n rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('$O/del_n$n.json')); print('   n=$n', round(d['value']), 'cw/s', d['config']['workload'])"
done
exit 0
