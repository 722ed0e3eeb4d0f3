#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload qary --steps 10 --warmup 3 --no-cpu > gpurun_out/bq7.json 2> gpurun_out/bq7.err; rc=$?; echo "bench qary rc=$rc"; [ $rc -eq 0 ] || exit $rc; python -c "
import json; d=json.load(open('gpurun_out/bq7.json')); print(round(d['value']/1e6,2), 'M frac', round(d['roofline']['frac'],4))"
timeout -k 10 600 python -u -m pytest tests/test_gpu_qary.py tests/test_gpu_fer.py -x -q --timeout 250 --timeout-method thread -k "qary or c4 or Qary or qsc" > gpurun_out/t7.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t7.log; [ $rc -eq 0 ] || exit $rc
