#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mc.py tests/test_gpu_fer.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t5.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t5.log; [ $rc -eq 0 ] || exit $rc
REPS=6 timeout -k 10 300 python -u scripts/mc_stages.py 262144 1048576 > gpurun_out/e2e5.txt 2>&1; rc=$?; grep median gpurun_out/e2e5.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/b5.json 2> gpurun_out/b5.err; rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.load(open('gpurun_out/b5.json')); print(round(d['value']/1e6,2), 'M frac', round(d['roofline']['frac'],4), 'e2e', d['mc_end_to_end'])"
