#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_tr.py > gpurun_out/ab_tr2.txt 2>&1; rc=$?; echo "ab rc=$rc"; tail -3 gpurun_out/ab_tr2.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_mc.py tests/test_gpu_leaf.py tests/test_gpu_prior.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t11.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t11.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/b11_$i.json 2> gpurun_out/b11_$i.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc; python -c "
import json; d=json.load(open('gpurun_out/b11_$i.json')); print(round(d['value']/1e6,2), 'M frac', round(d['roofline']['frac'],4), 'e2e', round(d['mc_end_to_end']['value']/1e6,2))"; done
