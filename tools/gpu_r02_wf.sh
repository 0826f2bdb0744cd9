#!/bin/bash
# Round 2: the wavefront loop (MODE 4) - parity with it forced on, its SIMD
# efficiency, and A/B against the lockstep kernel (and the pre-refactor base).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02wf}; O=$R/gpurun_out/$T; mkdir -p $O
cd $R
ZRT_WF=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_runtime.py -x -q --timeout 150 --timeout-method thread > $O/tests_wf.log 2>&1 || { tail -30 $O/tests_wf.log; exit 1; }
tail -2 $O/tests_wf.log
ZRT_WF=1 timeout -k 10 300 python -u tools/simd_eff.py 2:2048:2048:16 3:1024:1024:16 6:4096:4096:4 > $O/eff_wf.jsonl 2> $O/eff_wf.err || { tail -5 $O/eff_wf.err; exit 1; }
cat $O/eff_wf.jsonl
bash $R/tools/gpu_ab2.sh $T/c3 1 base=base lock=default wf=default:ZRT_WF=1 wf16=default:ZRT_WF=1,ZRT_WF_THRESH=16 wf48=default:ZRT_WF=1,ZRT_WF_THRESH=48 -- --scene 3 --width 1024 --height 1024 --spp 256 --steps 2 --warmup 1 || exit 1
bash $R/tools/gpu_ab2.sh $T/c5 1 lock=default wf=default:ZRT_WF=1 wf16=default:ZRT_WF=1,ZRT_WF_THRESH=16 -- --scene 6 --width 4096 --height 4096 --spp 64 --steps 2 --warmup 1 || exit 1
bash $R/tools/gpu_ab2.sh $T/c4 1 base=base lock=default wf=default:ZRT_WF=1 -- --steps 3 --warmup 1 || exit 1
