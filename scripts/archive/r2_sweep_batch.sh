#!/bin/bash
# Batch-size sweep of the headline decode, other alphabets of the q-ary kernel, the SCL line.
set -u
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/bsweep
cd $R
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
for spec in "b16:--batch 65536" "b18:--batch 262144" "b20:--batch 1048576" "b22:--batch 4194304" \
            "q2:--workload qary --q 2" "q3:--workload qary --q 3" "q8:--workload qary --q 8" "scl:--workload scl"; do
  name=${spec%%:*}; extra=${spec#*:}
  timeout -k 10 300 python bench.py $extra --steps 5 --warmup 2 --no-cpu --no-e2e > gpurun_out/bsweep/$name.json 2> gpurun_out/bsweep/$name.err
  rc=$?; echo "$name rc=$rc $(python -c "import json; d=json.load(open('gpurun_out/bsweep/$name.json')); print('%.3fM cw/s %.2f ms frac %.3f %s' % (d['value']/1e6, d['roofline']['kernel_ms'], d['roofline']['frac'], d['config'].get('workload')))")"
  [ $rc -eq 0 ] || { tail -3 gpurun_out/bsweep/$name.err; exit $rc; }
done
exit 0
