#!/bin/bash
# Round 2 (session 6): HEAD revalidation (GPU suite + driver bench command, C4),
# then C5-substitute A/B: wavefront loop at 4 (default) vs 5 waves/SIMD.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02s6}; O=$R/gpurun_out/$T; mkdir -p $O
cd $R
bash tools/gpu_r02_reentry.sh $T/reentry || exit 1
bash tools/gpu_ab2.sh $T/c5ab 2 wf4=default wf5=wf5 -- --scene 6 --width 4096 --height 4096 --spp 64 --steps 2 --warmup 1
