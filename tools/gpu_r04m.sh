#!/bin/bash
# GPU box, round 4: the full GPU suite on the 6-wave lockstep build; C5 A/B of
# the guard branch, FMA slabs and LDS attenuation rows of the path pool; a
# PMC set of C5 on the default build (write budget, HBM fraction).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04m; mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab.sh r04m/c5 2 default noguard nofma prow2 prow5 -- --scene 6 --width 4096 --height 4096 --spp 1024 --depth 20 --steps 1 --warmup 1 || exit 1
bash tools/gpu_pmc.sh r04m/c5pmc --scene 6 --width 4096 --height 4096 --spp 1024 --depth 20 --steps 1 --warmup 1 || exit 1
echo session-done
