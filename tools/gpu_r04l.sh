#!/bin/bash
# GPU box, round 4: waves per SIMD once attenuation codes freed registers:
# lockstep FAST 5/6/7 (C4, C3), path pool 4/5 (C5), list loops 6/7/8 (C2).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04l; mkdir -p $O
cd $R
export TMPDIR=/tmp
bash tools/ab.sh r04l/c4 2 default w6 w7 -- --no-reference-check || exit 1
bash tools/ab.sh r04l/c3 2 default w6 w7 -- --no-reference-check --scene 3 --width 1024 --height 1024 --spp 256 --depth 20 || exit 1
bash tools/ab.sh r04l/c2 2 default list7 list8 -- --no-reference-check --scene 1 --width 1000 --height 1000 --spp 1000 --depth 30 || exit 1
bash tools/ab.sh r04l/c5 2 default pool5 -- --no-reference-check --scene 6 --width 4096 --height 4096 --spp 1024 --depth 20 --steps 1 --warmup 1 || exit 1
echo session-done
