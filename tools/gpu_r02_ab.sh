#!/bin/bash
# Round 2 kernel A/B: GPU suite on the working tree's kernel, then interleaved
# bench A/B (default = working tree, prev = the last commit's kernel) on C4, C3
# and a reduced C5 substitute.  usage: bash tools/gpu_r02_ab.sh <tag> [variants...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02ab}; shift; V=${@:-default prev}; O=$R/gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab.sh $T/c4 2 $V -- --steps 5 --warmup 2 --no-reference-check || exit 1
bash tools/ab.sh $T/c3 2 $V -- --scene 3 --width 1024 --height 1024 --spp 256 --steps 5 --warmup 2 --no-reference-check || exit 1
bash tools/ab.sh $T/c5 1 $V -- --scene 6 --width 2048 --height 2048 --spp 256 --steps 3 --warmup 1 --no-reference-check || exit 1
