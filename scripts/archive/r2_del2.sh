#!/bin/bash
# Deletion measurement: fp64 VALU ceilings, the n=12 bench line, SQ + HBM counters at n=8 and n=10.
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 120 ./build/valu_peak > gpurun_out/valu_peak.json 2> gpurun_out/valu_peak.err
rc=$?; echo "valu_peak rc=$rc $(cat gpurun_out/valu_peak.json)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload deletion --n 12 --batch 32768 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_del_n12.json 2> gpurun_out/bench_del_n12.err
rc=$?; echo "bench del n12 rc=$rc"; cat gpurun_out/bench_del_n12.json | cut -c1-400; [ $rc -eq 0 ] || { tail -3 gpurun_out/bench_del_n12.err; exit $rc; }
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD"
SQ2="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR"
TAG=del_n8_r2b ARGS="--workload deletion" PASSES="$SQ1;$SQ2;FETCH_SIZE;WRITE_SIZE" bash scripts/prof_passes.sh || exit 1
TAG=del_n10_r2b ARGS="--workload deletion --n 10 --batch 65536" PASSES="$SQ1;$SQ2;FETCH_SIZE;WRITE_SIZE" bash scripts/prof_passes.sh || exit 1
exit 0
