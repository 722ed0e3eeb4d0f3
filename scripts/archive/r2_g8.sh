#!/bin/bash
# DPP lane exchanges (xor 4 / 8): correctness, decode + deletion parity, G=8/16 variant sweep.
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 60 ./build/dpptest || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_deletion.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_g8.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_g8.log; [ $rc -eq 0 ] || exit $rc
CASES="17:0 19:0 20:0 21:0 23:0" bash scripts/sweep.sh || exit 1
mkdir -p gpurun_out/n12 && CASES="17:0 19:0 20:0 21:0" BENCH_EXTRA="--n 12" bash scripts/sweep.sh || exit 1
exit 0
