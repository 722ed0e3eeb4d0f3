#!/bin/bash
# Decode parity for the listed binary variants, then one bench line each (decode only).
# usage: VARIANTS="24 26" N=10 [TESTK="26 or 27"] bash scripts/bench_variants.sh
set -u
mkdir -p gpurun_out
if [ -n "${TESTK:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py -k "$TESTK" -x -q --timeout 120 --timeout-method thread > gpurun_out/tv.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tv.log; [ $rc -eq 0 ] || exit $rc
fi
for v in ${VARIANTS:-24}; do
  timeout -k 10 200 python bench.py --steps ${STEPS:-10} --warmup 3 --n ${N:-10} --batch ${BATCH:-1048576} --variant $v --no-cpu --no-e2e ${BENCH_EXTRA:-} > gpurun_out/bv$v.json 2> gpurun_out/bv$v.err || { echo "bench v$v failed"; tail -3 gpurun_out/bv$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bv$v.json')); print('v$v', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],3), 'ms frac', round(d['roofline']['frac'],4))"
done
