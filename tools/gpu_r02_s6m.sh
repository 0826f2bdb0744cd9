#!/bin/bash
# Round 2 (session 6): C4 cost of the grazing margins' t-proportional term (norel: A/B only, inexact).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02s6m}
cd $R
bash tools/gpu_ab2.sh $T/c4ab 2 slack=default norel=norel noslack=noslack -- --steps 10 --warmup 3
