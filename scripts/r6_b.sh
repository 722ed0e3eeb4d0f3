#!/bin/bash
# Round 6: the whole GPU suite (code-length-specialised twins now the default at N = 1024 / 4096),
# the fixed-n A/B at C2 / C3, deletion bench lines after the guard-band scan change, the per-lane
# deletion kernel at n = 12 under occupancy caps, and the C5 profile.
# usage: OUT=r6b bash scripts/r6_b.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6b}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ab_fixed_n.py --n 10 > $O/ab_fixed_n10.txt 2>&1; rc=$?; cat $O/ab_fixed_n10.txt | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ab_fixed_n.py --n 12 --rounds 4 > $O/ab_fixed_n12.txt 2>&1; rc=$?; cat $O/ab_fixed_n12.txt | tail -3; [ $rc -eq 0 ] || exit $rc
run() {  # tag, args
  timeout -k 10 400 python3 bench.py $2 > $O/$1.json 2> $O/$1.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench $1 rc=$rc"; tail -3 $O/$1.err; return $rc; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('$1', round(d['value']/1e6,4), 'M  frac', round(d['roofline']['frac'],4))"
}
run c2 "--steps 10 --warmup 3 --no-cpu" || exit 1
for rep in 1 2; do
  run c5_$rep "--workload deletion --steps 10 --warmup 3 --no-cpu" || exit 1
  run c5k64_$rep "--workload deletion --del-k 64 --steps 10 --warmup 3 --no-cpu" || exit 1
  run d10_$rep "--workload deletion --n 10 --steps 5 --warmup 2 --no-cpu" || exit 1
done
run d11 "--workload deletion --n 11 --batch 262144 --steps 5 --warmup 2 --no-cpu" || exit 1
for cap in 0 4 2 1; do
  run d12_cap$cap "--workload deletion --n 12 --batch 32768 --steps 2 --warmup 1 --no-cpu --del-cap $cap" || exit 1
done
WL=deletion TAG=${OUT:-r6b}/del_n8_n02_dense EXTRA="" bash scripts/prof_sq.sh || exit 1
exit 0
