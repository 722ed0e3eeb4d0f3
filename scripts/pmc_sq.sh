#!/bin/bash
# SQ/GRBM counter passes on the decode kernel (one pass per group; each pass its own run).
# usage: GROUPS_FILE-free: PASSES="A,B,C;D,E" DECODE_EXTRA="--variant 17" bash scripts/pmc_sq.sh
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
python -c "import __graft_entry__ as g; g.build()" > $R/gpurun_out/build.log 2>&1 || exit 1
if [ -n "${LIST:-}" ]; then
  timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1; echo "list rc=$?"
fi
IFS=';' read -ra P <<< "${PASSES}"
i=0
for grp in "${P[@]}"; do
  i=$((i+1))
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc ${grp//,/ } --output-format csv -d $R/gpurun_out/sq_${TAG:-x}_$i -o pmc -- python3 ${PROFILED:-$R/scripts/decode_only.py --batch ${BATCH:-1048576} --reps 1 ${DECODE_EXTRA:-}} > $R/gpurun_out/sq_${TAG:-x}_$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; cd $R
  [ $rc -eq 0 ] || exit $rc
done
exit 0
