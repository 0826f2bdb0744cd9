#!/bin/bash
# Round 2: GPU tests at HEAD, then C5-substitute A/B (4096^2 x 64 spp):
# lockstep interval (ZRT_SYNC) and one tree copy vs the eight octant copies.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-r02c5ab}; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash $R/tools/gpu_ab2.sh ${1:-r02c5ab}/ab 1 s1=default s2=default:ZRT_SYNC=2 s4=default:ZRT_SYNC=4 s32=default:ZRT_SYNC=32 noentry=noentry oct1=oct1 \
  -- --scene 6 --width 4096 --height 4096 --spp 64 --steps 2 --warmup 1
