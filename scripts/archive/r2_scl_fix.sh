#!/bin/bash
# SCL at the bench's shape after the stack-limit fix: the default limit first (no kernel), then
# growing batches (64, 1024, 2048 resident workgroups), each its own process and time limit;
# the first failure ends the run.
set -u
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/scl
timeout -k 10 120 python -c "
import ctypes, sys; sys.path.insert(0, '.')
import torch
from polarcub_amd import _lib
L = _lib.lib(); L.pcub_scl_stack_limit.restype = ctypes.c_longlong
torch.cuda.init(); torch.zeros(1, device='cuda')
print('default stack limit', L.pcub_scl_stack_limit())
" || exit 1
for B in 4096 65536 1048576; do
  timeout -k 10 200 python -u scripts/dbg/scl_ladder.py $B || exit 1
done
timeout -k 10 300 python bench.py --workload scl --steps 3 --warmup 1 --no-cpu --no-e2e > gpurun_out/scl/bench.json 2> gpurun_out/scl/bench.err || { tail -3 gpurun_out/scl/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/scl/bench.json')); print('scl %.3fM cw/s %.2f ms fer %.4f' % (d['value']/1e6, d['roofline']['kernel_ms'], d['fer']))"
