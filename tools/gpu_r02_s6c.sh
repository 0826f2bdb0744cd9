#!/bin/bash
# Round 2 (session 6): grazing-ray fix (per-ray absolute slack in the narrowed culls):
# GPU suite, grazing diagnostics, A/B of the slack's cost (C4, C3, C5 substitute).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02s6c}; O=$R/gpurun_out/$T; mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/grazing_diag.py $O/grazing.json 3 0 4 2 > $O/grazing.log 2>&1 || { tail -20 $O/grazing.log; exit 1; }
grep -v amdgpu.ids $O/grazing.log
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|Error" $O/tests.log | head -20; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab2.sh $T/c4ab 2 slack=default noslack=noslack -- --steps 10 --warmup 3 || exit 1
bash tools/gpu_ab2.sh $T/c3ab 2 slack=default noslack=noslack -- --scene 3 --width 1024 --height 1024 --spp 256 --steps 5 --warmup 2 || exit 1
bash tools/gpu_ab2.sh $T/c5ab 1 slack=default noslack=noslack -- --scene 6 --width 4096 --height 4096 --spp 64 --steps 2 --warmup 1
