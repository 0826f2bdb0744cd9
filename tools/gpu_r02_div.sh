#!/bin/bash
# Round 2: short correctly rounded divisions.  GPU parity suite on the new kernel,
# then interleaved A/B (default = short divisions, slowdiv = HIP's IEEE `/`) on C4,
# C3 and C2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02div}; O=$R/gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab.sh $T/c4 2 default divonly slowdiv -- --steps 5 --warmup 2 --no-reference-check || exit 1
bash tools/ab.sh $T/c3 2 default divonly slowdiv -- --scene 3 --width 1024 --height 1024 --spp 256 --steps 5 --warmup 2 --no-reference-check || exit 1
bash tools/ab.sh $T/c2 1 default divonly slowdiv -- --scene 1 --width 1000 --height 1000 --spp 1000 --depth 30 --steps 3 --warmup 1 --no-reference-check || exit 1
