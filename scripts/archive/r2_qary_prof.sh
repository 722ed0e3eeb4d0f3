#!/bin/bash
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
timeout -k 10 300 python bench.py --workload qary --qsc-p 0.1100000001 --qregs 4 --qvariant 1 --steps 10 --warmup 3 --no-cpu > gpurun_out/bench_qary_standin.json 2>/dev/null
echo "stand-in frozen set: $(python -c "import json; d=json.load(open('gpurun_out/bench_qary_standin.json')); print('%.1fM cw/s %.2f ms' % (d['value']/1e6, d['roofline']['kernel_ms']))")"
TAG=qary_q4_s4v1 ARGS="--workload qary --qregs 4 --qvariant 1" PASSES="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY;SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT" bash scripts/prof_passes.sh || exit 1
exit 0
