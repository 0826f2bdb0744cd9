#!/bin/bash
# GPU box, round 4: the lockstep loop's RNG state and chunk sums kept in LDS
# (default) against VGPRs (nolst, the previous build): lockstep parity tests, C4
# and C3 interleaved, C4 write traffic.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04r; mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "loops_bit_exact or scanline or c3 or c2_matches or schedule or probe or xoshiro or prng or chunk or per_axis" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab.sh r04r/c4 2 default nolst -- --no-reference-check || exit 1
bash tools/ab.sh r04r/c3 2 default nolst -- --no-reference-check --scene 3 --width 1024 --height 1024 --spp 256 --depth 20 || exit 1
bash tools/gpu_pmc.sh r04r/pmc_c4 || exit 1
echo session-done
