#!/bin/bash
# Round 2 evidence, part 2: the C5 substitute at its full config (4096^2 x 4096
# spp) with rocprofv3 kernel trace and PMC passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02final2}; O=$R/gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
cd $R
bash $R/tools/gpu_pmc.sh $T/c5pmc --scene 6 --width 4096 --height 4096 --spp 4096 --steps 1 --warmup 1 || exit 1
python -c "import json; d=json.load(open('$O/c5pmc/bench_traced.json')); print('C5', d['value'], d['ms_per_step'])"
