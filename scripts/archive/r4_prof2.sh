#!/bin/bash
# profile of the shipped C2 kernel (the tiled-root twin of variant 26)
set -u
WL=awgn TAG=bin_v26_n10 EXTRA="" bash scripts/prof_sq.sh || exit 1
