#!/bin/bash
# q-ary v2 session: GPU q-ary tests, bench lines at G=4/2/1, HBM + SQ passes of the default.
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_qary.py tests/test_qary_fixtures.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_qary.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_qary.log; [ $rc -eq 0 ] || exit $rc
for G in 4 2 1; do
  timeout -k 10 300 python bench.py --workload qary --qlanes $G --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_qary_g$G.json 2> gpurun_out/bench_qary_g$G.err
  rc=$?; echo "bench qary G=$G rc=$rc"; cat gpurun_out/bench_qary_g$G.json; [ $rc -eq 0 ] || exit $rc
done
for Q in 3 8; do
  timeout -k 10 300 python bench.py --workload qary --q $Q --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_qary_q$Q.json 2> gpurun_out/bench_qary_q$Q.err
  rc=$?; echo "bench qary q=$Q rc=$rc"; cut -c1-400 gpurun_out/bench_qary_q$Q.json; [ $rc -eq 0 ] || exit $rc
done
TAG=qary_q4_n8 ARGS="--workload qary" PASSES="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY" bash scripts/prof_passes.sh || exit 1
exit 0
