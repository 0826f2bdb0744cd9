#!/bin/bash
# Round 2 (session 6), final kernel with the grazing-ray slack: GPU suite, grazing
# diagnostics, C4 rocprofv3 evidence (trace + PMC passes), the driver's bench command,
# C5 / C3 cost A/B (noslack = the inexact round-2 kernel; nogrow / norel / noleaf: one part off).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02s6j}; O=$R/gpurun_out/$T; mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|Error" $O/tests.log | head -20; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/grazing_diag.py $O/grazing.json 3 0 4 2 > $O/grazing.log 2>&1 || { tail -20 $O/grazing.log; exit 1; }
grep -v amdgpu.ids $O/grazing.log
bash tools/gpu_pmc.sh $T/c4pmc || exit 1
cd $R
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4.json')); r=d['roofline']; print('C4', d['value'], d['ms_per_step'], r['bound'], r['frac'])"
bash tools/gpu_ab2.sh $T/c5ab 1 slack=default nogrow=nogrow norel=norel noleaf=noleaf noslack=noslack -- --scene 6 --width 4096 --height 4096 --spp 64 --steps 2 --warmup 1 || exit 1
bash tools/gpu_ab2.sh $T/c3ab 1 slack=default noslack=noslack -- --scene 3 --width 1024 --height 1024 --spp 256 --steps 5 --warmup 2
