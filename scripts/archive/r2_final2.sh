#!/bin/bash
# Final round-2 check: smoke + full GPU suite + bench lines, then the q-ary profile after the
# whole-round grid and SQ counters of the n = 8 deletion kernel.
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
bash scripts/r2_full.sh || exit $?
TAG=fin2_qary ARGS="--workload qary" PASSES="FETCH_SIZE;WRITE_SIZE" bash scripts/prof_passes.sh || exit 1
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_LDS"
TAG=fin2_del_n8 ARGS="--workload deletion" PASSES="FETCH_SIZE;WRITE_SIZE;$SQ;SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" bash scripts/prof_passes.sh || exit 1
exit 0
