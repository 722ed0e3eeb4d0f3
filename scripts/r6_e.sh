#!/bin/bash
# Round 6: the binary decode's wave tiles from a counter vs the static stride (A/B at C2 and C3's
# shape), then the whole GPU suite.
# usage: OUT=r6e bash scripts/r6_e.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6e}
mkdir -p $O
timeout -k 10 300 python3 scripts/ab_dyn_tiles.py --n 10 > $O/ab_dyn10.txt 2>&1; rc=$?; tail -3 $O/ab_dyn10.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/ab_dyn_tiles.py --n 12 --rounds 4 > $O/ab_dyn12.txt 2>&1; rc=$?; tail -3 $O/ab_dyn12.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 > $O/c2.json 2> $O/c2.err; rc=$?; echo "bench rc=$rc"
python3 -c "import json; d=json.load(open('$O/c2.json')); print('c2', round(d['value']/1e6,3), d['mc_end_to_end']['value']/1e6)"
exit 0
