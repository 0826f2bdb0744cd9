#!/bin/bash
# C4 (and C3) bench A/B of build variants, no test suite.  usage: bash tools/gpu_r02_ab_c4.sh <tag> <variants...>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; shift
cd $R
bash tools/ab.sh $T/c4 2 "$@" -- --steps 5 --warmup 2 --no-reference-check || exit 1
bash tools/ab.sh $T/c3 1 "$@" -- --scene 3 --width 1024 --height 1024 --spp 256 --steps 5 --warmup 2 --no-reference-check || exit 1
