#!/bin/bash
# rocprofv3 on one bench workload's decode step: a kernel-trace/stats run, then each PMC
# group in its own run and time limit (never combined with any trace domain).
#   TAG=del_n8 ARGS="--workload deletion" PASSES="A B C;D E" bash scripts/prof_passes.sh
# Output: gpurun_out/$TAG/{trace,pmc1,pmc2,...}
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:?}
mkdir -p $O
ARGS=${ARGS:-}
cd /tmp
if [ -z "${NO_TRACE:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/scripts/profile_step.py $ARGS --reps ${REPS:-5} > $O/trace.log 2>&1
  rc=$?; echo "trace $TAG rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/trace.log; exit $rc; }
fi
IFS=';' read -ra P <<< "${PASSES:-FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum}"
i=0
for grp in "${P[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $O/pmc$i -o pmc -- python3 $R/scripts/profile_step.py $ARGS --reps 1 > $O/pmc$i.log 2>&1
  rc=$?; echo "pmc $TAG pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/pmc$i.log; exit $rc; }
done
exit 0
