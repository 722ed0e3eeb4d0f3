#!/bin/bash
# Round 6 diagnostics of the n0 = 4 wave kernel: the same launches with the tasks skipped
# (pcub_sc_set_deletion_wave(3)), so the difference is the tasks' share.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6w4x}
mkdir -p $O
cd $R
run() {  # tag, args
  timeout -k 10 300 python3 bench.py $2 > $O/$1.json 2> $O/$1.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench $1 rc=$rc"; tail -3 $O/$1.err; return $rc; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('$1', round(d['value']/1e3,2), 'k cw/s  kernel', d['roofline'].get('kernel'), round(d['roofline'].get('kernel_ms',0),2), 'ms')"
}
run d12 "--workload deletion --n 12 --batch 32768 --steps 3 --warmup 1 --no-cpu" || exit 1
run d12_notask "--workload deletion --n 12 --batch 32768 --steps 3 --warmup 1 --no-cpu --del-wave 3" || exit 1
run d13_notask "--workload deletion --n 13 --batch 16384 --steps 3 --warmup 1 --no-cpu --del-wave 3" || exit 1
run d14_notask "--workload deletion --n 14 --batch 8192 --steps 3 --warmup 1 --no-cpu --del-wave 3" || exit 1
exit 0
