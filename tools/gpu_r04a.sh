#!/bin/bash
# GPU box, round 4 first session: the grazing-triangle probe on the current
# kernel (pre-fix counts), the lockstep interval A/B for the list
# loop (C2) and the bunny (C4), then the GPU test suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04a; mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/grazing_tris_probe.py $O/grazing_probe.json 20000 > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cat $O/probe.log
bash tools/gpu_env_ab.sh r04a/sync_c2 2 "ZRT_SYNC=1" "ZRT_SYNC=32" "ZRT_SYNC=4" -- --scene 1 --width 1000 --height 1000 --spp 1000 --depth 30 || exit 1
bash tools/gpu_env_ab.sh r04a/sync_c4 2 "ZRT_SYNC=1" "ZRT_SYNC=2" -- --no-reference-check || exit 1
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not grazing_triangles" > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
exit $rc
