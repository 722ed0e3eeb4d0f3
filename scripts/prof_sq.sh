#!/bin/bash
# Kernel trace + HBM traffic + SQ instruction-mix passes of one bench workload, each pass its own
# run and kill-timeout, into gpurun_out/<TAG>/ in the layout scripts/collect_profiles.py reads.
# usage: WL=awgn TAG=bin_v26_n10 EXTRA="--variant 26" [SQ=0] bash scripts/prof_sq.sh
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:?}
mkdir -p $O
B="python3 $R/bench.py --workload ${WL:?} --no-cpu --no-e2e ${EXTRA:-}"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- $B --steps 3 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "trace $TAG rc=$rc"; [ $rc -eq 0 ] || exit $rc
GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum")
if [ "${SQ:-1}" = 1 ]; then
  GROUPS_+=("SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU")
  GROUPS_+=("SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS SQ_INSTS_VMEM")
  GROUPS_+=("SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS")
  GROUPS_+=("GRBM_GUI_ACTIVE GRBM_COUNT")
fi
for grp in "${GROUPS_[@]}"; do
  tag=${grp%% *}
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$tag -o pmc -- $B --steps 1 --warmup 0 > $O/pmc_$tag.log 2>&1
  rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
