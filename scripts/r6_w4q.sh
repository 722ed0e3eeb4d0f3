#!/bin/bash
# Round 6: quick A/B of the n0 = 4 wave kernel at n = 12 (wave tests, then bench lines).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6w4q}
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_deletion.py \
  -k "wave_kernel or wide_shapes or 4-11-0 or 4-12-0" > $O/pytest.log 2>&1; rc=$?
tail -1 $O/pytest.log; [ $rc -eq 0 ] || { tail -30 $O/pytest.log; exit $rc; }
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --workload deletion --n 12 --batch 32768 --steps 3 --warmup 1 --no-cpu > $O/d12_$rep.json 2> $O/d12_$rep.err || exit 1
  python3 -c "import json; d=json.load(open('$O/d12_$rep.json')); print('d12', round(d['value']/1e3,2), 'k')"
done
exit 0
