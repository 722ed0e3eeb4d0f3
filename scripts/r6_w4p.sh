#!/bin/bash
# Round 6: kernel trace + HBM + SQ passes of the final n0 = 4 wave kernel at n = 12 (8192 codewords).
set -u
R=$GRAFT_REPO_ROOT
WL=deletion TAG=${OUT:-r6w4p}/del_n12_w4 EXTRA="--n 12 --batch 8192" bash $R/scripts/prof_sq.sh || exit 1
exit 0
