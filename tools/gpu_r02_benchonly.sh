#!/bin/bash
# The driver's bench command (C4) and the C5 bench line after the PMC entries of
# the current kernel are merged (their roofline / write budget read them).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02bench}; O=$R/gpurun_out/$T; mkdir -p $O
cd $R
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4.json')); r=d['roofline']; print('C4', d['value'], d['ms_per_step'], r['bound'], r['frac'], r.get('write_budget'))"
timeout -k 10 600 python bench.py --scene 6 --width 4096 --height 4096 --spp 4096 --steps 1 --warmup 1 > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/c5.json')); r=d['roofline']; print('C5', d['value'], d['ms_per_step'], r['bound'], r['frac'], r.get('write_budget'))"
