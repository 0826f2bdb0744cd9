#!/bin/bash
# GPU box, round 4: the full GPU suite on the 6-wave lockstep build; C5 A/B of
# the guard branch, FMA slabs, LDS attenuation rows and the sample-gated (hybrid)
# pool; C3 on the pool with and without the gate against lockstep; C4 lockstep
# interval (ZRT_SYNC); a PMC set of C5 on the default build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04n; mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
C5="--scene 6 --width 4096 --height 4096 --spp 1024 --depth 20 --steps 1 --warmup 1"
C3="--no-reference-check --scene 3 --width 1024 --height 1024 --spp 256 --depth 20"
bash tools/ab.sh r04n/c5 2 default noguard nofma prow2 prow5 gate gates -- $C5 || exit 1
bash tools/ab.sh r04n/c3lock 2 default -- $C3 || exit 1
ZRT_POOL=1 bash tools/ab.sh r04n/c3pool 2 default gate gates -- $C3 || exit 1
bash tools/gpu_env_ab.sh r04n/c4sync 2 "ZRT_SYNC=1" "ZRT_SYNC=2" "ZRT_SYNC=4" -- --no-reference-check || exit 1
bash tools/gpu_pmc.sh r04n/c5pmc $C5 || exit 1
echo session-done
