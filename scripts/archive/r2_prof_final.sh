#!/bin/bash
# Round-2 final profiles of the default kernels: kernel trace + HBM + SQ passes for the
# headline (N = 1024), N = 4096, q-ary C4 and deletion n = 10 (n0 = 3).
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_LDS"
TAG=fin_bin_n10 ARGS="--workload awgn" PASSES="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;$SQ" bash scripts/prof_passes.sh || exit 1
TAG=fin_bin_n12 ARGS="--workload awgn --n 12" PASSES="FETCH_SIZE;WRITE_SIZE" bash scripts/prof_passes.sh || exit 1
TAG=fin_qary ARGS="--workload qary" PASSES="FETCH_SIZE;WRITE_SIZE;$SQ" bash scripts/prof_passes.sh || exit 1
TAG=fin_del_n10 ARGS="--workload deletion --n 10 --batch 65536" PASSES="FETCH_SIZE;WRITE_SIZE;$SQ" bash scripts/prof_passes.sh || exit 1
exit 0
