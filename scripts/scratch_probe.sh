#!/bin/bash
# n0 = 4 deletion (n = 12): is the private-segment kernel's occupancy capped by the runtime's scratch limit?
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/scratch_probe; mkdir -p $O
A="--workload deletion --n 12 --batch 65536 --steps 2 --warmup 1 --no-cpu --no-e2e"
timeout -k 10 200 python3 bench.py $A > $O/default.json 2> $O/default.err || exit $?
python3 -c "import json; d=json.load(open('$O/default.json')); print('default', d['value'], d['ms_per_step'])"
HSA_SCRATCH_SINGLE_LIMIT=34359738368 timeout -k 10 200 python3 bench.py $A > $O/big.json 2> $O/big.err || exit $?
python3 -c "import json; d=json.load(open('$O/big.json')); print('limit 32G', d['value'], d['ms_per_step'])"
