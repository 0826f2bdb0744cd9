#!/bin/bash
# GPU box, round 4: C5 on one tree copy (planes selected per ray; the 8 octant
# copies are 8x the footprint of a million-triangle tree) and the pool's shade
# threshold on the current kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04p; mkdir -p $O
cd $R
export TMPDIR=/tmp
C5="--scene 6 --width 4096 --height 4096 --spp 1024 --depth 20 --steps 1 --warmup 1"
bash tools/ab.sh r04p/c5 2 default oct1 -- $C5 || exit 1
bash tools/gpu_env_ab.sh r04p/thresh 1 "ZRT_WF_THRESH=40" "ZRT_WF_THRESH=48" "ZRT_WF_THRESH=56" -- $C5 || exit 1
bash tools/ab.sh r04p/c3 1 default oct1 -- --no-reference-check --scene 3 --width 1024 --height 1024 --spp 256 --depth 20 || exit 1
echo session-done
