#!/bin/bash
# rocprofv3 passes on the decode kernel: kernel-trace stats, then one PMC group per pass.
# usage: TAG=r1 ARGS="--n 10 --batch 1048576" bash scripts/prof_pmc.sh
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${TAG:-run}
ARGS=${ARGS:-}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
python -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/scripts/decode_only.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace failed"; tail $OUT/trace.log; exit 1; }
i=0
for grp in ${PMC_GROUPS:-"FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"} ${EXTRA_PMC:-}; do
  grp=${grp//,/ }
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o pmc -- python3 $R/scripts/decode_only.py $ARGS --reps 1 > $OUT/pmc$i.log 2>&1 || { echo "pmc $grp failed"; tail -5 $OUT/pmc$i.log; }
done
echo done
