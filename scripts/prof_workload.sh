#!/bin/bash
# Kernel-trace stats + HBM counter passes (FETCH_SIZE, WRITE_SIZE, L2 hit/miss) of one
# bench workload, each pass its own run and time limit, into gpurun_out/<tag>/ in the
# layout scripts/collect_profiles.py reads (--src gpurun_out/<tag>).
# usage: WL=deletion TAG=del_n8_n02 EXTRA="" bash scripts/prof_workload.sh
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:?}
mkdir -p $O
python -c "import __graft_entry__ as g; g.build()" > $O/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --workload ${WL:?} --steps 3 --warmup 1 --no-cpu ${EXTRA:-} > $O/prof.log 2>&1
rc=$?; echo "prof $TAG rc=$rc"; [ $rc -eq 0 ] || exit $rc
for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  tag=${grp%% *}
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$tag -o pmc -- python3 $R/bench.py --workload $WL --steps 1 --warmup 0 --no-cpu ${EXTRA:-} > $O/pmc_$tag.log 2>&1
  rc=$?; echo "pmc $grp rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
