#!/bin/bash
# Round 5, re-entry check: smoke and the GPU suite on a library rebuilt from the committed sources,
# the C2 headline line, and the list decoder at the large shape the ABI advertises (q = 4,
# N = 4096, L = 32) at the largest grid its slab allows, with a kernel trace.
# usage: OUT=r5f4 bash scripts/r5_final4.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r5f4}
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > $O/c2.json 2> $O/c2.err; rc=$?; echo "bench c2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
cat $O/c2.json
timeout -k 10 300 python3 bench.py --workload scl --steps 3 --warmup 1 --batch 65536 > $O/scl_n8_L8.json 2> $O/scl_n8_L8.err
rc=$?; echo "bench scl n8 rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof_scl_n12 -o scl -- \
  python3 $R/bench.py --workload scl --n 12 --list-size 32 --batch 32768 --steps 1 --warmup 0 --no-cpu \
  > $O/scl_n12_L32.json 2> $O/scl_n12_L32.err
rc=$?; echo "bench scl n12 L32 rc=$rc"; cat $O/scl_n12_L32.json; exit $rc
