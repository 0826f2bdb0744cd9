#!/bin/bash
# Round 2 (session 6): which part of the grazing-ray slack costs C5 / C3 (A/B-only inexact variants).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02s6i}; O=$R/gpurun_out/$T; mkdir -p $O
cd $R
bash tools/gpu_ab2.sh $T/c5ab 1 slack=default nogrow=nogrow norel=norel noleaf=noleaf noslack=noslack -- --scene 6 --width 4096 --height 4096 --spp 64 --steps 2 --warmup 1 || exit 1
bash tools/gpu_ab2.sh $T/c3ab 1 slack=default nogrow=nogrow norel=norel noleaf=noleaf noslack=noslack -- --scene 3 --width 1024 --height 1024 --spp 256 --steps 5 --warmup 2
