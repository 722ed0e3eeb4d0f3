#!/bin/bash
# Link A/B experiment kernels into the in-tree library without touching the library build.
#   bash scripts/exp_build.sh <dir>
# <dir>/inc<N>/ (or <dir>/inc/) holds experiment N's modified copies of csrc headers (searched before
# csrc/), <dir>/kx<N>.flags its extra compiler flags (optional), <dir>/kx*.hip the experiment
# translation units: each defines its kernels in its own namespace (#define pcub pcubxN before including
# sc_bin_kern.h) and an extern "C" pcub_exp_kernel_N(int v, int compact).  This script writes the
# dispatcher pcub_exp_kernel(e, v, compact) -> pcub_exp_kernel_<e>, compiles everything for gfx950 and
# relinks polarcub_amd/lib/libpolarcub_hip.so from the library's objects plus these, and removes the
# library's stamp so that the next `python -m polarcub_amd.build` relinks the clean library.
set -eu
D=$(cd "$1" && pwd)
R=$(cd "$(dirname "$0")/.." && pwd)
CS=$R/polarcub_amd/csrc
FL="--offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -fPIC -std=c++17"
N=$(ls $D/kx*.hip | wc -l)
{
  echo 'extern "C" {'
  for f in $D/kx*.hip; do e=$(basename $f .hip); e=${e#kx}; echo "void* pcub_exp_kernel_$e(int v, int compact);"; done
  echo 'void* pcub_exp_kernel(int e, int v, int compact) {'
  echo '    switch (e) {'
  for f in $D/kx*.hip; do e=$(basename $f .hip); e=${e#kx}; echo "        case $e: return pcub_exp_kernel_$e(v, compact);"; done
  echo '        default: return nullptr;'
  echo '    }'
  echo '}'
  echo '}'
} > $D/dispatch.cpp
pids=()
[ "${SKIP_COMPILE:-0}" = 1 ] || for f in $D/kx*.hip; do
  e=$(basename $f .hip); e=${e#kx}; INC=$D/inc$e; [ -d $INC ] || INC=$D/inc
  XF=""; [ -f ${f%.hip}.flags ] && XF=$(cat ${f%.hip}.flags)  # extra compiler flags of experiment N
  /opt/rocm/bin/hipcc $FL $XF -I$INC -I$R/include -I$CS -c $f -o ${f%.hip}.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
g++ -O2 -fPIC -c $D/dispatch.cpp -o $D/dispatch.o
python3 - "$R" "$D" <<'PY'
import subprocess, sys, glob, os
R, D = sys.argv[1], sys.argv[2]
sys.path.insert(0, R)
from polarcub_amd import build as b
objs = [b._obj(s) for s in b.SOURCES] + sorted(glob.glob(os.path.join(D, "kx*.o"))) + [os.path.join(D, "dispatch.o")]
subprocess.run([b.HIPCC, "--offload-arch=" + b.ARCH, "-shared", "-fPIC"] + objs + ["-o", b.LIB + ".tmp"], check=True)
os.replace(b.LIB + ".tmp", b.LIB)
if os.path.exists(b.LIB + ".sha256"):
    os.remove(b.LIB + ".sha256")  # the next library build relinks without the experiments
print("linked", len(objs), "objects")
PY
