#!/bin/bash
# Round 6: decode variants at N = 1024 / 4096 (G = 8 split variants 30 / 33 and variant 31 with its new
# tiled-root twin), and the end-to-end Monte-Carlo at 2^18- and 2^20-codeword chunks.
# usage: OUT=r6var bash scripts/r6_var.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6var}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q -k "26 or 31" --timeout 250 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, args
  timeout -k 10 300 python3 bench.py $2 > $O/$1.json 2> $O/$1.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench $1 rc=$rc"; tail -3 $O/$1.err; return $rc; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); e=d.get('mc_end_to_end',{}); print('$1', round(d['value']/1e6,2), 'M  e2e', round(e.get('value',0)/1e6,2))"
}
run c2_v26 "--steps 10 --warmup 3 --no-cpu" || exit 1
run c2_v26_e2e20 "--steps 10 --warmup 3 --no-cpu --e2e-chunk 1048576" || exit 1
run c2_v30 "--steps 10 --warmup 3 --no-cpu --no-e2e --variant 30" || exit 1
run c2_v33 "--steps 10 --warmup 3 --no-cpu --no-e2e --variant 33" || exit 1
run c3_v31 "--n 12 --steps 5 --warmup 2 --no-cpu --no-e2e" || exit 1
run c3_v30 "--n 12 --steps 5 --warmup 2 --no-cpu --no-e2e --variant 30" || exit 1
run c3_v33 "--n 12 --steps 5 --warmup 2 --no-cpu --no-e2e --variant 33" || exit 1
run c3_v31b "--n 12 --steps 5 --warmup 2 --no-cpu --no-e2e" || exit 1
timeout -k 10 300 python3 scripts/mc_stages.py 262144 1048576 > $O/mc_stages.txt 2>&1; echo "mc_stages rc=$?"; tail -15 $O/mc_stages.txt
exit 0
