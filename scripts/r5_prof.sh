#!/bin/bash
# Round 5 profiles of the shipped kernels (kernel trace + HBM + SQ passes, scripts/prof_sq.sh):
# C2 (variant 26 tiled root), C3's N = 4096 (variant 31), C4, the deletion n0 = 4 kernel at n = 12.
set -u
WL=awgn TAG=bin_v26_n10 EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=awgn TAG=bin_v31_n12 EXTRA="--n 12" bash scripts/prof_sq.sh || exit 1
WL=qary TAG=qary_q4_n8 EXTRA="" bash scripts/prof_sq.sh || exit 1
WL=deletion TAG=del_n12_n04 EXTRA="--n 12 --batch 16384" SQ=1 bash scripts/prof_sq.sh || exit 1
exit 0
