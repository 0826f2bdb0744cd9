#!/bin/bash
# Round 2 evidence run on the current kernel: GPU suite, the driver's bench
# command, rocprofv3 kernel trace of the bench, C2/C3 lines, C5 at its full
# config with PMC passes (tools/gpu_pmc.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02final}; O=$R/gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4.json')); print('C4', d['value'], d['ms_per_step'], d['roofline']['bound'], d['roofline']['frac'])"
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4trace -o run -- python $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-reference-check > $O/c4_traced.json 2> $O/c4_traced.err || { tail -5 $O/c4_traced.err; exit 1; }
cd $R
timeout -k 10 400 python bench.py --scene 1 --width 1000 --height 1000 --spp 1000 --depth 30 > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 400 python bench.py --scene 3 --width 1024 --height 1024 --spp 256 --depth 20 > $O/c3.json 2> $O/c3.err || exit 1
python -c "
import json
for c in ('c2','c3'):
    d=json.load(open('$O/'+c+'.json')); print(c, d['value'], d['ms_per_step'])"
bash $R/tools/gpu_pmc.sh $T/c5pmc --scene 6 --width 4096 --height 4096 --spp 4096 --steps 1 --warmup 1 || exit 1
python -c "import json; d=json.load(open('$O/c5pmc/bench_traced.json')); print('C5', d['value'], d['ms_per_step'])"
