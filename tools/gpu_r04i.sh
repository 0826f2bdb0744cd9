#!/bin/bash
# GPU box, round 4: C5 A/B of the FMA slabs (1024 spp), then the tiled-4K frame
# (scene 2 at 4096x4096 @ 64 spp) at N = 1, 2, 3 over gloo on one GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04i; mkdir -p $O
cd $R
export TMPDIR=/tmp
bash tools/ab.sh r04i/c5 2 default nofma -- --scene 6 --width 4096 --height 4096 --spp 1024 --depth 20 --steps 1 --warmup 1 || exit 1
bash tools/gpu_rehearse_dist.sh r04i/dist4k 4k || exit 1
echo session-done
