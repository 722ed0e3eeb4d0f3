#!/bin/bash
# PMC passes (one rocprofv3 run per pass, each under its own kill-timeout) over a profiled command.
# usage: TAG=x PASSES="A B C;D E" CMD="scripts/decode_only.py --batch 1048576 --reps 1" bash scripts/pmc_passes.sh
# The library must already be built in-tree (it is not rebuilt here).
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:?}
mkdir -p $O
IFS=';' read -ra P <<< "${PASSES:?}"
i=0
for grp in "${P[@]}"; do
  i=$((i+1))
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$i -o pmc -- python3 $R/${CMD:?} > $O/pmc_$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; cd $R
  [ $rc -eq 0 ] || exit $rc
done
exit 0
