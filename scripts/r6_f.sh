#!/bin/bash
# Round 6: work tiles from a counter in the q-ary and deletion decodes too -- the whole GPU suite, then
# each BASELINE shape with counter tiles and with the static stride (--static-tiles), interleaved.
# usage: OUT=r6f bash scripts/r6_f.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6f}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, args
  timeout -k 10 400 python3 bench.py $2 > $O/$1.json 2> $O/$1.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench $1 rc=$rc"; tail -3 $O/$1.err; return $rc; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); e=d.get('mc_end_to_end',{}); print('$1', round(d['value']/1e6,4), 'M  frac', round(d['roofline']['frac'],4), ' e2e', round(e.get('value',0)/1e6,2))"
}
for rep in 1 2; do
  for m in dyn static; do
    X=""; [ $m = static ] && X="--static-tiles"
    run c4_${m}_$rep "--workload qary --steps 10 --warmup 3 --no-cpu $X" || exit 1
    run c5_${m}_$rep "--workload deletion --steps 10 --warmup 3 --no-cpu $X" || exit 1
    run c5k64_${m}_$rep "--workload deletion --del-k 64 --steps 10 --warmup 3 --no-cpu $X" || exit 1
    run d10_${m}_$rep "--workload deletion --n 10 --steps 5 --warmup 2 --no-cpu $X" || exit 1
  done
done
run c2 "--steps 10 --warmup 3" || exit 1
run c3 "--n 12 --steps 5 --warmup 2 --no-cpu" || exit 1
exit 0
