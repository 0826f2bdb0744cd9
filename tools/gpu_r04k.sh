#!/bin/bash
# GPU box, round 4: attenuation rows decoded in pairs (default) against one at a
# time (nopairs) on C5; the lockstep FAST kernel at 6 waves/SIMD (w6) on C4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04k; mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "scene4 or c5_substitute or texel or loops_bit_exact or guard or c2_matches" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab.sh r04k/c5 2 default nopairs -- --scene 6 --width 4096 --height 4096 --spp 1024 --depth 20 --steps 1 --warmup 1 || exit 1
bash tools/ab.sh r04k/c4 2 default w6 -- --no-reference-check || exit 1
echo session-done
