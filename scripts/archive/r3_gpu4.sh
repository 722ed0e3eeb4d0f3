#!/bin/bash
# round 3: compact MC pipeline parity, bench with end-to-end line, flat-private diagnostic, profiles
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mc.py tests/test_gpu_decode.py tests/test_gpu_qary.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t4.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/t4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
python -c "
import json; d = json.load(open('gpurun_out/bench.json')); print('C2', round(d['value']/1e6, 2), 'M frac', round(d['roofline']['frac'], 4), 'e2e', round(d['mc_end_to_end']['value']/1e6, 2), 'M cpu', round(d['cpu_baseline']['value']/1e6, 3))"
timeout -k 10 120 ./scripts/dbg/flat_private; echo "flat_private rc=$?"
WL=qary TAG=qary_q4_n8 EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=deletion TAG=del_n8_n02 EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=deletion TAG=del_n8_n02_k64 EXTRA="--del-k 64" bash scripts/prof_sq.sh || exit 1
WL=awgn TAG=bin_v26_n10 EXTRA="--n 10" bash scripts/prof_sq.sh || exit 1
