#!/bin/bash
# Bench sweep: "variant:max_blocks" pairs from $CASES, decode-only bench lines (no CPU leg).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -20 gpurun_out/build.log; exit 1; }
for c in ${CASES}; do
  v=${c%%:*}; m=${c##*:}
  timeout -k 10 ${T_BENCH:-300} python bench.py --steps ${STEPS:-5} --warmup 2 --variant $v --max-blocks $m --no-cpu ${BENCH_EXTRA:-} > gpurun_out/sw_${v}_${m}.json 2> gpurun_out/sw_err.log
  rc=$?
  python -c "import json,sys; r=json.loads(open('gpurun_out/sw_${v}_${m}.json').read()); print('v=$v m=$m %.2fM cw/s kern %.2f ms frac %.3f fer %.4f' % (r['value']/1e6, r['roofline']['kernel_ms'], r['roofline']['frac'], r['fer']))" || { echo "case $c rc=$rc"; tail -5 gpurun_out/sw_err.log; }
  [ $rc -eq 0 ] || exit $rc
done
exit 0
