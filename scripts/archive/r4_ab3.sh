#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_tr.py > gpurun_out/ab_tr.txt 2>&1; rc=$?; echo "ab rc=$rc"; tail -4 gpurun_out/ab_tr.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_mc.py -x -q --timeout 250 --timeout-method thread > gpurun_out/t9.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t9.log; [ $rc -eq 0 ] || exit $rc
