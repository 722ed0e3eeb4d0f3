#!/bin/bash
# Round 6 checkpoint: smoke, the whole GPU suite, bench lines (C2 default; C3 shape's new default;
# C4 with the S = 4 and S = 8 split levels; N = 16384 variant 17 vs 33).
# usage: OUT=r6chk bash scripts/r6_check.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6chk}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, args
  timeout -k 10 400 python3 bench.py $2 > $O/$1.json 2> $O/$1.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench $1 rc=$rc"; tail -3 $O/$1.err; return $rc; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); e=d.get('mc_end_to_end',{}); print('$1', round(d['value']/1e6,3), 'M  frac', round(d['roofline']['frac'],4), ' e2e', round(e.get('value',0)/1e6,2), d['config'].get('kernel_variant',''))"
}
run c2 "--steps 10 --warmup 3" || exit 1
run c3 "--n 12 --steps 5 --warmup 2 --no-cpu" || exit 1
for rep in 1 2; do
  run c4_s4_$rep "--workload qary --steps 10 --warmup 3 --no-cpu --no-e2e" || exit 1
  run c4_s8_$rep "--workload qary --steps 10 --warmup 3 --no-cpu --no-e2e --qregs 8" || exit 1
done
for rep in 1 2; do
  run c5_$rep "--workload deletion --steps 10 --warmup 3 --no-cpu" || exit 1
  run c5k64_$rep "--workload deletion --del-k 64 --steps 10 --warmup 3 --no-cpu" || exit 1
done
run d10 "--workload deletion --n 10 --steps 5 --warmup 2 --no-cpu" || exit 1
run n14_v17 "--n 14 --batch 131072 --steps 3 --warmup 1 --no-cpu --no-e2e" || exit 1
run n14_v33 "--n 14 --batch 131072 --steps 3 --warmup 1 --no-cpu --no-e2e --variant 33" || exit 1
WL=deletion TAG=${OUT:-r6chk}/del_n8_n02_dense EXTRA="" bash scripts/prof_sq.sh || exit 1
exit 0
