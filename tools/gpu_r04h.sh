#!/bin/bash
# GPU box, round 4: C5 A/B - default (texel values by division, guard code in the
# pool kernel) against the build without the guard code; textured parity tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04h; mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "scene4 or c5_substitute or texel or loops_bit_exact or guard" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab.sh r04h/c5 1 default noguard -- --scene 6 --width 4096 --height 4096 --spp 1024 --depth 20 --steps 1 --warmup 1 || exit 1
bash tools/ab.sh r04h/c4 1 default noguard -- --no-reference-check || exit 1
echo session-done
