#!/bin/bash
# GPU box, round 4: the per-axis grazing guard after its fixes (loose_slot widened,
# exact hazard entries): the probe and C3 cost (path-pool loop) at several
# coefficients; C4 without the guard.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04e; mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "(trace_ or loops_bit_exact) and not grazing_triangles" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C3="--scene 3 --width 1024 --height 1024 --spp 256 --depth 20 --no-reference-check"
for g in 0.000061035 0.00024414 0.0009765625; do
  ZRT_GUARD_K=$g timeout -k 10 600 python -u tools/grazing_tris_probe.py $O/probe_$g.json 20000 > $O/probe_$g.log 2>&1 || { tail -20 $O/probe_$g.log; exit 1; }
  echo "guard $g"; grep -v amdgpu.ids $O/probe_$g.log
done
bash tools/gpu_env_ab.sh r04e/c4 2 "ZRT_GUARD_K=0" -- --no-reference-check || exit 1
bash tools/gpu_env_ab.sh r04e/c3 1 "ZRT_GUARD_K=0" "ZRT_POOL=1" "ZRT_GUARD_K=0.000061035" "ZRT_GUARD_K=0.00024414" "ZRT_GUARD_K=0.0009765625" -- $C3 || exit 1
echo session-done
