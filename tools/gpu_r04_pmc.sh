#!/bin/bash
# GPU box, round 4 final build: rocprofv3 PMC sets (tools/gpu_pmc.sh) of configs
# C4, C3, C2 and C5 (4096 spp, the config), after one C5 A/B of scalar node loads
# in the path pool.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=r04final
cd $R
export TMPDIR=/tmp
bash tools/ab.sh $T/c5_poolscalar 1 default poolscalar -- --scene 6 --width 4096 --height 4096 --spp 1024 --depth 20 --steps 1 --warmup 1 || exit 1
bash tools/gpu_pmc.sh $T/pmc_c4 || exit 1
bash tools/gpu_pmc.sh $T/pmc_c3 --scene 3 --width 1024 --height 1024 --spp 256 --depth 20 || exit 1
bash tools/gpu_pmc.sh $T/pmc_c2 --scene 1 --width 1000 --height 1000 --spp 1000 --depth 30 || exit 1
bash tools/gpu_pmc.sh $T/pmc_c5 --scene 6 --width 4096 --height 4096 --spp 4096 --depth 20 --steps 1 --warmup 1 || exit 1
echo session-done
