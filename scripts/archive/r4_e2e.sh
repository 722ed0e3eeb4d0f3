#!/bin/bash
# e2e pipeline: chunk sizes, overlapped and serial, with spread
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
true
PCUB_MC_SERIAL=1 REPS=6 timeout -k 10 300 python -u scripts/mc_stages.py 524288 262144 > gpurun_out/e2e_serial.txt 2>&1; rc=$?; grep median gpurun_out/e2e_serial.txt; [ $rc -eq 0 ] || exit $rc
REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/e2e_prof -o e2e -- python3 scripts/mc_stages.py 1048576 > gpurun_out/e2e_prof.txt 2>&1; rc=$?; echo "prof rc=$rc"
find gpurun_out/e2e_prof -name '*kernel_stats.csv' | head -1 | xargs cut -d, -f1-4 | head -12
