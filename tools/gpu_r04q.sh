#!/bin/bash
# GPU box: the scene-6 grazing-triangle test, then the final PMC sets.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04final; mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 380 --timeout-method thread \
  -k "grazing_triangles_c5" > $O/grazing_c5.log 2>&1
rc=$?; tail -3 $O/grazing_c5.log; [ $rc -le 1 ] || exit 1
bash tools/gpu_r04_pmc.sh
