#!/bin/bash
# round 4 GPU session 2: smoke, the changed GPU tests, the default bench line
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_mc.py tests/test_gpu_fer.py tests/test_gpu_deletion.py tests/test_abi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t2.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
