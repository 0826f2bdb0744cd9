#!/bin/bash
# Round 2 evidence on the current kernel, part 1: GPU suite, the driver's bench
# command (C4), its rocprofv3 kernel trace + PMC passes (tools/gpu_pmc.sh), C3
# and C2 bench lines.  Part 2 (C5 at its full config + PMC): tools/gpu_r02_final2_c5.sh.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02final2}; O=$R/gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4.json')); print('C4', d['value'], d['ms_per_step'], d['kernel_ms_avg'])"
bash $R/tools/gpu_pmc.sh $T/c4pmc --steps 5 --warmup 1 || exit 1
cd $R
timeout -k 10 400 python bench.py --scene 3 --width 1024 --height 1024 --spp 256 --depth 20 > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 400 python bench.py --scene 1 --width 1000 --height 1000 --spp 1000 --depth 30 > $O/c2.json 2> $O/c2.err || exit 1
python -c "
import json
for c in ('c2','c3'):
    d=json.load(open('$O/'+c+'.json')); print(c, d['value'], d['ms_per_step'])"
