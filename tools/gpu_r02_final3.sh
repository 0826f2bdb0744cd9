#!/bin/bash
# Round 2: the driver's bench command again after the PMC entries of the
# current kernel were merged (profiles/latest_pmc.json), so its roofline and
# write budget read this kernel's counters; then the TD/TCP probe pre vs current.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02final3}; O=$R/gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4.json')); r=d['roofline']; print('C4', d['value'], d['ms_per_step'], r['bound'], r['frac'], r.get('write_budget'))"
bash $R/tools/gpu_r02_tdprobe.sh $T/td pre default || exit 1
