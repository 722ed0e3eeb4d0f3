#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_deletion.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t4.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/b4.json 2> gpurun_out/b4.err; rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.load(open('gpurun_out/b4.json')); print(round(d['value']/1e6,2), 'M frac', round(d['roofline']['frac'],4), 'e2e', d['mc_end_to_end']['value'])"
timeout -k 10 100 ./scripts/dbg/bin_phase 20 > gpurun_out/ph4.txt 2>&1; cat gpurun_out/ph4.txt
