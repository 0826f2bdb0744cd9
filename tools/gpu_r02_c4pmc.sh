#!/bin/bash
# Round 2: the current FAST kernel on C4 - STATS counters at the full size, PMC passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02c4c}; O=$R/gpurun_out/$T; mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/simd_eff.py 2:2048:2048:1024 > $O/eff.jsonl 2> $O/eff.err || { tail -5 $O/eff.err; exit 1; }
cat $O/eff.jsonl
bash $R/tools/gpu_pmc.sh $T/pmc || exit 1
