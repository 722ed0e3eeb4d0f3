#!/bin/bash
# round 3: short division in f/g -- full GPU parity, bench lines, deletion re-profile
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t3.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="26 24" N=10 bash scripts/bench_variants.sh || exit 1
VARIANTS="24 31" N=12 BATCH=262144 bash scripts/bench_variants.sh || exit 1
timeout -k 10 300 python bench.py --workload qary --steps 5 --warmup 2 --no-cpu > gpurun_out/bq.json 2> gpurun_out/bq.err || exit 1
timeout -k 10 300 python bench.py --workload deletion --steps 5 --warmup 2 --no-cpu > gpurun_out/bd.json 2> gpurun_out/bd.err || exit 1
timeout -k 10 300 python bench.py --workload deletion --del-k 64 --steps 5 --warmup 2 --no-cpu > gpurun_out/bd64.json 2> gpurun_out/bd64.err || exit 1
python -c "
import json
for f in ('bq', 'bd', 'bd64'):
    d = json.load(open('gpurun_out/%s.json' % f)); print(f, round(d['value']/1e6, 2), 'M', d.get('fer'), d['roofline']['kernel_ms'])
"
WL=deletion TAG=del_n8_n02 EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=deletion TAG=del_n8_n02_k64 EXTRA="--del-k 64" bash scripts/prof_sq.sh || exit 1
WL=awgn TAG=bin_v26_n10 EXTRA="--n 10" bash scripts/prof_sq.sh || exit 1
