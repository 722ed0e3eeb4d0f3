#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_deletion.py -x -q -k "wide" --timeout 250 --timeout-method thread > gpurun_out/t6a.log 2>&1; rc=$?; echo "wide rc=$rc"; tail -3 gpurun_out/t6a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload qary --steps 10 --warmup 3 --no-cpu > gpurun_out/bq6.json 2> gpurun_out/bq6.err; rc=$?; echo "bench qary rc=$rc"; [ $rc -eq 0 ] || exit $rc; python -c "
import json; d=json.load(open('gpurun_out/bq6.json')); print(round(d['value']/1e6,2), 'M frac', round(d['roofline']['frac'],4))"
timeout -k 10 700 python -u -m pytest tests/test_gpu_mc.py tests/test_gpu_deletion.py tests/test_gpu_qary.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t6.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t6.log; [ $rc -eq 0 ] || exit $rc
for n in 12 13 14; do timeout -k 10 300 python bench.py --workload deletion --n $n --batch 4096 --steps 2 --warmup 1 --no-cpu > gpurun_out/bdel_n$n.json 2> gpurun_out/bdel_n$n.err; rc=$?; echo "bench n=$n rc=$rc"; [ $rc -eq 0 ] || exit $rc; python -c "
import json; d=json.load(open('gpurun_out/bdel_n$n.json')); print(d['config']['workload'], round(d['value'],1), 'cw/s', d['roofline']['kernel'])"; done
