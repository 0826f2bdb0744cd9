#!/bin/bash
# GPU box, round 4: the path pool without the guard branch (MODE 5; guarded renders
# MODE 7) and its global attenuation rows path-major (default) vs row-major; a PMC
# set of C5 on the default build (write budget).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04o; mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "pool or c5_substitute or loops_bit_exact or guard or grazing or texel or scanline" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C5="--scene 6 --width 4096 --height 4096 --spp 1024 --depth 20 --steps 1 --warmup 1"
bash tools/ab.sh r04o/c5 3 default rowmajor -- $C5 || exit 1
bash tools/gpu_pmc.sh r04o/c5pmc $C5 || exit 1
echo session-done
