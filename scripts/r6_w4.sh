#!/bin/bash
# Round 6: the n0 = 4 wave-per-task deletion kernel (sc_del_w4.hip): parity, then bench lines at
# n = 12, 13, 14 against the lane-per-trellis kernel, and (PROF=1) a profile at n = 12.
# usage: OUT=r6w4 [TESTS=all|w4] [PROF=1] bash scripts/r6_w4.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6w4}
mkdir -p $O
cd $R
run() {  # tag, args
  timeout -k 10 300 python3 bench.py $2 > $O/$1.json 2> $O/$1.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench $1 rc=$rc"; tail -3 $O/$1.err; return $rc; }
  python3 -c "import json; d=json.load(open('$O/$1.json')); print('$1', round(d['value']/1e3,2), 'k cw/s  kernel', d['roofline'].get('kernel'), round(d['roofline'].get('kernel_ms',0),2), 'ms  fer', d.get('fer'))"
}
if [ "${TESTS:-w4}" = all ]; then K="wave_kernel or wide_shapes or random_vs_oracle or edge_golden"; else K="wave_kernel or wide_shapes or 4-11-0 or 4-12-0"; fi
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_deletion.py \
  -k "$K" > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/pytest.log | tail -3; [ $rc -eq 0 ] || { tail -30 $O/pytest.log; exit $rc; }
run d12 "--workload deletion --n 12 --batch 32768 --steps 3 --warmup 1 --no-cpu" || exit 1
run d13 "--workload deletion --n 13 --batch 16384 --steps 3 --warmup 1 --no-cpu" || exit 1
run d13w "--workload deletion --n 13 --batch 16384 --steps 3 --warmup 1 --no-cpu --del-wave 2" || exit 1
run d14 "--workload deletion --n 14 --batch 8192 --steps 3 --warmup 1 --no-cpu" || exit 1
run d14w "--workload deletion --n 14 --batch 8192 --steps 3 --warmup 1 --no-cpu --del-wave 2" || exit 1
if [ "${PROF:-0}" = 1 ]; then
  WL=deletion TAG=${OUT:-r6w4}/del_n12_w4 EXTRA="--n 12 --batch 8192" bash scripts/prof_sq.sh || exit 1
fi
exit 0
