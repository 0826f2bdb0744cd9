#!/bin/bash
# Round 2 (session 6): the grazing-exact kernel on the full C5-substitute config and on C3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02s6l}; O=$R/gpurun_out/$T; mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --scene 3 --width 1024 --height 1024 --spp 256 --steps 5 --warmup 2 > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
timeout -k 10 600 python bench.py --scene 6 --width 4096 --height 4096 --spp 4096 --depth 20 --steps 2 --warmup 1 --no-cpu-baseline --no-reference-check > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
for c in c3 c5; do python -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['bound'], d['roofline']['frac'])"; done
