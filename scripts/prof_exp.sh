#!/bin/bash
# Kernel trace + HBM + SQ instruction-mix passes of scripts/decode_only.py (C2 workload by default),
# each pass its own run and kill-timeout, into gpurun_out/<TAG>/ (the layout collect_profiles.py reads).
# usage: TAG=x2_n10 ARGS="--exp 2" bash scripts/prof_exp.sh
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:?}
mkdir -p $O
B="python3 $R/scripts/decode_only.py ${ARGS:-}"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- $B --reps 4 > $O/prof.log 2>&1
rc=$?; echo "trace $TAG rc=$rc"; [ $rc -eq 0 ] || exit $rc
GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum")
GROUPS_+=("SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU")
GROUPS_+=("SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS SQ_INSTS_VMEM")
GROUPS_+=("SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS")
GROUPS_+=("GRBM_GUI_ACTIVE GRBM_COUNT")
for grp in "${GROUPS_[@]}"; do
  tag=${grp%% *}
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$tag -o pmc -- $B --reps 1 > $O/pmc_$tag.log 2>&1
  rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
