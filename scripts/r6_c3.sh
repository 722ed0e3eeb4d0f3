#!/bin/bash
# Round 6: the binary decode suite with the G = 8 split variants, C3-shape bench lines (N = 2048 /
# 4096 / 8192, G = 4 vs G = 8 split), the N = 4096 G = 8 kernel's profile, and the Monte-Carlo
# pipeline's stage times (kernel trace).
# usage: OUT=r6c3 bash scripts/r6_c3.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6c3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_edge_long.py -x -q --timeout 250 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, args
  timeout -k 10 300 python3 bench.py $2 > $O/$1.json 2> $O/$1.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench $1 rc=$rc"; tail -3 $O/$1.err; return $rc; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('$1', round(d['value']/1e6,3), 'M variant', d['config'].get('kernel_variant'))"
}
for rep in 1 2; do
  run n11_v26_$rep "--n 11 --steps 5 --warmup 2 --no-cpu --no-e2e" || exit 1
  run n11_v30_$rep "--n 11 --steps 5 --warmup 2 --no-cpu --no-e2e --variant 30" || exit 1
  run n12_v31_$rep "--n 12 --steps 5 --warmup 2 --no-cpu --no-e2e --variant 31" || exit 1
  run n12_v30_$rep "--n 12 --steps 5 --warmup 2 --no-cpu --no-e2e --variant 30" || exit 1
  run n13_v31_$rep "--n 13 --batch 262144 --steps 5 --warmup 2 --no-cpu --no-e2e --variant 31" || exit 1
  run n13_v33_$rep "--n 13 --batch 262144 --steps 5 --warmup 2 --no-cpu --no-e2e --variant 33" || exit 1
done
WL=awgn TAG=${OUT:-r6c3}/bin_v30_n12 EXTRA="--n 12 --variant 30" bash scripts/prof_sq.sh || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mcst -o run -- python3 $R/scripts/mc_stages.py 262144 > $O/mc_stages.txt 2>&1
echo "mc_stages rc=$?"; tail -4 $O/mc_stages.txt
exit 0
