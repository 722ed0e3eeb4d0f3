#!/bin/bash
# Round 5 profiles of the final kernels (kernel trace + HBM + SQ passes, scripts/prof_sq.sh).
set -u
WL=awgn TAG=bin_v26_n10 EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=qary TAG=qary_q4_n8 EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=deletion TAG=del_n8_n02_dense EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=deletion TAG=del_n8_n02_k64_dense EXTRA="--del-k 64" bash scripts/prof_sq.sh || exit 1
exit 0
