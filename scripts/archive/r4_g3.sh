#!/bin/bash
# round 4 GPU session 3: q-ary tiled + MC + FER tests; awgn / qary / deletion bench lines
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_qary.py tests/test_gpu_mc.py tests/test_gpu_fer.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t3.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/t3.log; [ $rc -eq 0 ] || exit $rc
for wl in awgn qary deletion; do
  timeout -k 10 400 python bench.py --workload $wl --steps 10 --warmup 3 > gpurun_out/b_$wl.json 2> gpurun_out/b_$wl.err; rc=$?; echo "bench $wl rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/b_$wl.err; exit $rc; }
  python -c "
import json; d=json.load(open('gpurun_out/b_$wl.json'))
print('$wl', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],3), 'ms frac', round(d['roofline']['frac'],4), 'fer', d.get('fer'), 'e2e', d.get('mc_end_to_end',{}).get('value'), 'cpu', d['cpu_baseline']['value'])"
done
