#!/bin/bash
set -u
mkdir -p gpurun_out
for i in 1 2; do
for b in ab_orig ab_new; do timeout -k 10 100 ./scripts/dbg/$b 20 99 > gpurun_out/$b.$i.txt 2>&1; rc=$?; echo "$b rc=$rc $(grep tiles gpurun_out/$b.$i.txt)"; [ $rc -eq 0 ] || exit $rc; done
done
