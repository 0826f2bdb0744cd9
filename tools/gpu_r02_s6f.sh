#!/bin/bash
# Round 2 (session 6): where the grazing-ray fix costs: grown inner boxes vs the leaf slots' slack (C4, C5 substitute).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02s6f}; O=$R/gpurun_out/$T; mkdir -p $O
cd $R
bash tools/gpu_ab2.sh $T/c4ab 1 slack=default noleaf=noleaf nogrow=nogrow noslack=noslack -- --steps 10 --warmup 3 || exit 1
bash tools/gpu_ab2.sh $T/c5ab 1 slack=default noleaf=noleaf nogrow=nogrow noslack=noslack -- --scene 6 --width 4096 --height 4096 --spp 64 --steps 2 --warmup 1
