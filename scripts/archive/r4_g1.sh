#!/bin/bash
# round 4, GPU session 1: binary decode parity (all variants) + deletion table checks + the large SCL shape, then variant bench lines
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_deletion.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tdec.log 2>&1; rc=$?; echo "pytest dec/del rc=$rc"; tail -3 gpurun_out/tdec.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="26 33 34 35" bash scripts/bench_variants.sh || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_scl.py -x -v --timeout 280 --timeout-method thread -k n4096 > gpurun_out/tscl.log 2>&1; rc=$?; echo "pytest scl rc=$rc"; tail -3 gpurun_out/tscl.log; [ $rc -eq 0 ] || exit $rc
