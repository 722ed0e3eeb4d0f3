#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_qtr.py > gpurun_out/ab_qtr.txt 2>&1; rc=$?; echo "ab rc=$rc"; tail -4 gpurun_out/ab_qtr.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_qary.py tests/test_gpu_mc.py tests/test_gpu_fer.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t10.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t10.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload qary --steps 10 --warmup 3 --no-cpu > gpurun_out/bq10.json 2> gpurun_out/bq10.err; rc=$?; echo "bench qary rc=$rc"; [ $rc -eq 0 ] || exit $rc; python -c "
import json; d=json.load(open('gpurun_out/bq10.json')); print(round(d['value']/1e6,2), 'M frac', round(d['roofline']['frac'],4))"
