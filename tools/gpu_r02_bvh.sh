#!/bin/bash
# Round 2: full GPU suite (incl. the device BVH build), default bench, C5 line with preprocessing timings.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=${1:-r02bvh}; O=$R/gpurun_out/$T; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log; grep -E "device build" $O/tests.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
ZRT_DEBUG_LAUNCH=1 timeout -k 10 300 python bench.py --scene 6 --width 4096 --height 4096 --spp 256 --steps 2 --warmup 1 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { tail -5 $O/c5.err; exit 1; }
grep "zrt preprocess" $O/c5.err; python -c "import json; d=json.load(open('$O/c5.json')); print(d['value'], d['kernel_ms_avg'])"
