#!/bin/bash
# Round 6: kernel-trace passes over 10 timed + 3 warm-up steps (the bench's own step counts) for the
# shipped C2 / C3 / C4 / C5 kernels, so the profiled average is over warm launches like the bench's.
# usage: OUT=r6h bash scripts/r6_h.sh
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r6h}
mkdir -p $O
cd /tmp
for t in "bin_v26_n10:--workload awgn" "bin_v30_n12:--workload awgn --n 12" "qary_q4_n8:--workload qary" "del_n8_n02_dense:--workload deletion"; do
  tag=${t%%:*}; args=${t#*:}
  mkdir -p $O/$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag/prof -o run -- python3 $R/bench.py $args --no-cpu --no-e2e --steps 10 --warmup 3 > $O/$tag/prof.log 2>&1
  rc=$?; echo "trace $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
