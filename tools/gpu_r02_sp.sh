#!/bin/bash
# Round 2: scalar-cache reads of wave-uniform primitives - parity, then A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02sp}; O=$R/gpurun_out/$T; mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash $R/tools/gpu_ab2.sh $T/c4 2 sp0=sp0 sp=sp new=default -- --steps 3 --warmup 1 --no-cpu-baseline || exit 1
bash $R/tools/gpu_ab2.sh $T/c3 1 sp0=sp0 sp=sp new=default -- --scene 3 --width 1024 --height 1024 --spp 256 --steps 2 --warmup 1 || exit 1
bash $R/tools/gpu_ab2.sh $T/c5 1 sp0=sp0 sp=sp new=default -- --scene 6 --width 4096 --height 4096 --spp 64 --steps 2 --warmup 1 || exit 1
