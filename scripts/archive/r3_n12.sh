#!/bin/bash
# round 3: N=4096 default -> variant 31 (split level, bits in scratch): tests, bench, profile
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_mc.py tests/test_gpu_facade.py -x -q --timeout 120 --timeout-method thread > gpurun_out/n12_test.log 2>&1
rc=$?; tail -3 gpurun_out/n12_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --n 12 --steps 5 --warmup 2 > gpurun_out/n12_bench.json 2> gpurun_out/n12_bench.err
rc=$?; cat gpurun_out/n12_bench.json; [ $rc -eq 0 ] || exit $rc
WL=awgn TAG=bin_v31_n12 EXTRA="--n 12" bash scripts/prof_sq.sh
