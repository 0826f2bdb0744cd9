#!/bin/bash
# Round 2 (session 6): grazing-ray mismatches per traversal (tools/grazing_diag.py),
# the driver's bench command (C4), C5-substitute A/B of the wavefront loop at 4 vs 5 waves/SIMD.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02s6b}; O=$R/gpurun_out/$T; mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/grazing_diag.py $O/grazing.json 3 0 4 2 > $O/grazing.log 2>&1 || { tail -20 $O/grazing.log; exit 1; }
cat $O/grazing.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4.json')); r=d['roofline']; print('C4', d['value'], d['ms_per_step'], r['bound'], r['frac'])"
bash tools/gpu_ab2.sh $T/c5ab 2 wf4=default wf5=wf5 -- --scene 6 --width 4096 --height 4096 --spp 64 --steps 2 --warmup 1
