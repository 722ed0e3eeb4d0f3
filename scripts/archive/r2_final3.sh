#!/bin/bash
# Round-2 closing check: smoke, the whole GPU suite, bench lines, and the n = 8 deletion profile
# of the shipped kernel (collapse over gathered paths) under its bench tag.
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
bash scripts/r2_full.sh || exit $?
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_BRANCH"
TAG=fin3_del_n8 ARGS="--workload deletion" PASSES="FETCH_SIZE;WRITE_SIZE;$SQ" bash scripts/prof_passes.sh || exit 1
exit 0
