#!/bin/bash
set -u
mkdir -p gpurun_out
for i in 1 2; do timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-e2e > gpurun_out/b8_$i.json 2> gpurun_out/b8_$i.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc; python -c "
import json; d=json.load(open('gpurun_out/b8_$i.json')); print(round(d['value']/1e6,2), 'M frac', round(d['roofline']['frac'],4))"; done
timeout -k 10 700 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_deletion.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t8.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t8.log; [ $rc -eq 0 ] || exit $rc
