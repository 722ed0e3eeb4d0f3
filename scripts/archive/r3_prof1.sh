#!/bin/bash
# round 3: instruction-mix profiles of the four bench kernels (binary N=1024 / 4096, q-ary C4, deletion C5)
set -u
R=$GRAFT_REPO_ROOT
WL=awgn TAG=bin_v26_n10 EXTRA="--n 10" bash $R/scripts/prof_sq.sh || exit 1
WL=awgn TAG=bin_n12 EXTRA="--n 12" bash $R/scripts/prof_sq.sh || exit 1
WL=qary TAG=qary_q4_n8 EXTRA="" bash $R/scripts/prof_sq.sh || exit 1
WL=deletion TAG=del_n8_n02 EXTRA="" bash $R/scripts/prof_sq.sh || exit 1
