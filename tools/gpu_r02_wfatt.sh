#!/bin/bash
# Wavefront loop LDS plan: GPU tests of the loops, then C5 (reduced) A/B of
# 4 attenuation rows in LDS (default) vs 2 (att2).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02wfatt}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "loops or c5 or multi or schedule" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab.sh $T/c5 2 default att2 -- --scene 6 --width 2048 --height 2048 --spp 256 --steps 3 --warmup 1 --no-reference-check || exit 1
