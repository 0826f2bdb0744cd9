#!/bin/bash
# GPU box, round 4 third session: the list loop with a per-wave unit pool (C2),
# and a leaf-only grazing margin (probe + cost).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04c; mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "not grazing_triangles" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C2="--scene 1 --width 1000 --height 1000 --spp 1000 --depth 30"
C3="--scene 3 --width 1024 --height 1024 --spp 256 --depth 20 --no-reference-check"
bash tools/gpu_env_ab.sh r04c/c2 2 "ZRT_LIST_LANES=1" "ZRT_LIST_LANES=0" -- $C2 || exit 1
for g in 0.00006103515625 0.0009765625 0.015625; do
  ZRT_GRAZE_LEAF=$g timeout -k 10 600 python -u tools/grazing_tris_probe.py $O/probe_leaf_$g.json 20000 > $O/probe_leaf_$g.log 2>&1 || { tail -20 $O/probe_leaf_$g.log; exit 1; }
  echo "graze_leaf $g"; grep -v amdgpu.ids $O/probe_leaf_$g.log
done
bash tools/gpu_env_ab.sh r04c/c3 1 "ZRT_GRAZE_LEAF=0" "ZRT_GRAZE_LEAF=0.00006103515625" "ZRT_GRAZE_LEAF=0.0009765625" "ZRT_GRAZE_LEAF=0.015625" -- $C3 || exit 1
bash tools/gpu_env_ab.sh r04c/c4 1 "ZRT_GRAZE_LEAF=0" "ZRT_GRAZE_LEAF=0.00006103515625" "ZRT_GRAZE_LEAF=0.0009765625" "ZRT_GRAZE_LEAF=0.015625" -- --no-reference-check || exit 1
echo session-done
