#!/bin/bash
# GPU box, round 4 second session: the GPU suite on the FMA-slab build, the list
# loop with per-lane work items (C2), FMA slabs against the reference's form
# (abvar/nofma), the grazing-margin coefficient's effect on the grazing-triangle
# probe and its cost on C3 / C4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04b; mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "not grazing_triangles" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C2="--scene 1 --width 1000 --height 1000 --spp 1000 --depth 30"
C3="--scene 3 --width 1024 --height 1024 --spp 256 --depth 20 --no-reference-check"
bash tools/gpu_env_ab.sh r04b/c2 2 "ZRT_LIST_LANES=1" "ZRT_LIST_LANES=0" -- $C2 || exit 1
bash tools/ab.sh r04b/fma_c4 2 default nofma -- --no-reference-check || exit 1
bash tools/ab.sh r04b/fma_c3 2 default nofma -- $C3 || exit 1
for g in 0 0.00006103515625 0.0009765625 0.015625; do
  ZRT_GRAZE_M=$g timeout -k 10 600 python -u tools/grazing_tris_probe.py $O/probe_$g.json 20000 > $O/probe_$g.log 2>&1 || { tail -20 $O/probe_$g.log; exit 1; }
  echo "graze_m $g"; grep -v amdgpu.ids $O/probe_$g.log
done
bash tools/gpu_env_ab.sh r04b/c3 1 "ZRT_GRAZE_M=0" "ZRT_GRAZE_M=0.00006103515625" "ZRT_GRAZE_M=0.0009765625" "ZRT_GRAZE_M=0.015625" -- $C3 || exit 1
bash tools/gpu_env_ab.sh r04b/c4 1 "ZRT_GRAZE_M=0" "ZRT_GRAZE_M=0.00006103515625" "ZRT_GRAZE_M=0.0009765625" "ZRT_GRAZE_M=0.015625" -- --no-reference-check || exit 1
echo session-done
# the full C3 frame with the REFERENCE traversal beside FAST (frame hashes)
timeout -k 10 900 python bench.py --scene 3 --width 1024 --height 1024 --spp 256 --depth 20 --no-cpu-baseline > $O/c3_ref.json 2> $O/c3_ref.err || { tail -5 $O/c3_ref.err; exit 1; }
python -c "import json; d=json.load(open('$O/c3_ref.json')); print('C3', d['value'], d['reference_traversal'])"
echo session-done-2
