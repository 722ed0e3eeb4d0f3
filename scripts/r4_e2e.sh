#!/bin/bash
# e2e pipeline: chunk sizes (serial at 2^20) with spread, then kernel stats of one serial pass
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
REPS=6 timeout -k 10 300 python -u scripts/mc_stages.py 1048576 262144 131072 > gpurun_out/e2e_chunks.txt 2>&1; rc=$?; cat gpurun_out/e2e_chunks.txt | grep median; [ $rc -eq 0 ] || exit $rc
REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/e2e_prof -o e2e -- python3 scripts/mc_stages.py 1048576 > gpurun_out/e2e_prof.txt 2>&1; rc=$?; echo "prof rc=$rc"
find gpurun_out/e2e_prof -name '*kernel_stats.csv' | head -1 | xargs cut -d, -f1-4 | head -12
