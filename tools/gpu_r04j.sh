#!/bin/bash
# GPU box, round 4: the path-pool loop with wave-uniform next nodes through the
# scalar cache (ZRT_POOL_SCALAR=1 build) against the default, on C3 (pool forced) and C5.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04j; mkdir -p $O
cd $R
export TMPDIR=/tmp
ZRT_POOL=1 bash tools/ab.sh r04j/c3 2 default poolscalar -- --scene 3 --width 1024 --height 1024 --spp 256 --depth 20 --no-reference-check || exit 1
bash tools/ab.sh r04j/c5 1 default poolscalar -- --scene 6 --width 4096 --height 4096 --spp 1024 --depth 20 --steps 1 --warmup 1 || exit 1
echo session-done
