#!/bin/bash
# Round 2: PMC passes (tools/gpu_pmc.sh) on the C5 substitute, lockstep loop vs
# the wavefront loop: what bounds the FAST kernel on a million-triangle mesh.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
A="--scene 6 --width 4096 --height 4096 --spp 16 --steps 2 --warmup 1"
ZRT_WF=0 bash $R/tools/gpu_pmc.sh r02c5pmc/lock $A || exit 1
ZRT_WF=1 bash $R/tools/gpu_pmc.sh r02c5pmc/wf $A || exit 1
bash $R/tools/gpu_ab2.sh r02c5pmc/ab 2 lock=default:ZRT_WF=0 wf=default:ZRT_WF=1 wf48=default:ZRT_WF=1,ZRT_WF_THRESH=48 wf56=default:ZRT_WF=1,ZRT_WF_THRESH=56 -- --scene 6 --width 4096 --height 4096 --spp 64 --steps 2 --warmup 1
