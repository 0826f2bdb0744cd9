#!/bin/bash
# Round 2 re-entry: HEAD revalidation - GPU suite and the driver's bench command (C4).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02reentry}; O=$R/gpurun_out/$T; mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4.json')); r=d['roofline']; print('C4', d['value'], d['ms_per_step'], r['bound'], r['frac'])"
