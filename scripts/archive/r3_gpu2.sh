#!/bin/bash
# round 3: new MC generators + decode parity of the new variants, then a variant sweep at N=1024 / 4096
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mc.py tests/test_gpu_decode.py tests/test_gpu_deletion.py tests/test_gpu_genie.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="26 30 32" N=10 bash scripts/bench_variants.sh || exit 1
VARIANTS="24 30 31" N=12 BATCH=262144 bash scripts/bench_variants.sh || exit 1
timeout -k 10 300 python bench.py --workload qary --steps 5 --warmup 2 --no-cpu > gpurun_out/bq.json 2> gpurun_out/bq.err || exit 1
timeout -k 10 300 python bench.py --workload deletion --steps 5 --warmup 2 --no-cpu > gpurun_out/bd.json 2> gpurun_out/bd.err || exit 1
python -c "
import json
for f in ('bq', 'bd'):
    d = json.load(open('gpurun_out/%s.json' % f)); print(f, round(d['value']/1e6, 2), 'M', d.get('fer'), d['data'][:60])
"
