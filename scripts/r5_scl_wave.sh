#!/bin/bash
# Round 5: list decoder wave mode (k_scl_wave) -- the SCL GPU tests (wave vs lane mode, oracle
# pins), then the N = 4096, L = 32 bench line in wave mode and the C4-shape line in lane mode.
# usage: OUT=r5scl bash scripts/r5_scl_wave.sh
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${OUT:-r5scl}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_scl.py tests/test_torch_ops.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_scl.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_scl.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --workload scl --n 12 --list-size 32 --batch 32768 --steps 1 --warmup 1 --no-cpu > $O/scl_n12_L32_wave.json 2> $O/scl_n12_L32_wave.err
rc=$?; echo "bench scl n12 L32 wave rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$O/scl_n12_L32_wave.json')); print(d['value'], d['ms_per_step'], d['fer'])"
timeout -k 10 300 python3 bench.py --workload scl --n 10 --list-size 8 --batch 65536 --steps 2 --warmup 1 --no-cpu > $O/scl_n10_L8_wave.json 2> $O/scl_n10_L8_wave.err
rc=$?; echo "bench scl n10 L8 wave rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$O/scl_n10_L8_wave.json')); print(d['value'], d['ms_per_step'], d['fer'])"
exit 0
