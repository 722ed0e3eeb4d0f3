#!/bin/bash
# Profile several binary decode variants back to back (trace + HBM + SQ passes each).
# usage: VARIANTS="24 26" N=10 bash scripts/prof_two.sh
set -u
for v in ${VARIANTS:-24}; do
  TAG=bin_v${v}_n${N:-10} ARGS="--n ${N:-10} --batch ${BATCH:-1048576} --variant $v" \
  EXTRA_PMC="SQ_WAVES,SQ_INSTS_VALU,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_ANY,SQ_INSTS_SALU GRBM_GUI_ACTIVE,GRBM_COUNT" \
  bash $GRAFT_REPO_ROOT/scripts/prof_pmc.sh || exit 1
done
