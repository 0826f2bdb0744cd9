#!/bin/bash
# C5-substitute probe: is the deep-tree (wavefront) loop bound by node bytes?
# default vs dblnode (every global wide-node read done twice, from another octant
# copy: twice the node bytes through TA/TD and the caches), at a reduced C5 size.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02c5probe}
cd $R
bash tools/ab.sh $T 2 default dblnode -- --scene 6 --width 2048 --height 2048 --spp 256 --steps 3 --warmup 1 --no-reference-check || exit 1
