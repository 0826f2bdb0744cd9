#!/bin/bash
# GPU box, round 4 final build: the full GPU suite, smoke, bench lines of C4 (with
# the CPU baseline and the REFERENCE-traversal frame), C3, C2, C5 (their rooflines
# from the PMC entries in profiles/latest_pmc.json), and the N-rank gloo
# rehearsals of C3 and of north_star's tiled 4K frame against the committed hashes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=r04final; O=$R/gpurun_out/$T; mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python bench.py > $O/c4.json 2> $O/c4.err || { echo "bench c4 failed"; tail -5 $O/c4.err; exit 1; }
timeout -k 10 300 python bench.py --scene 3 --width 1024 --height 1024 --spp 256 --depth 20 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { echo "bench c3 failed"; exit 1; }
timeout -k 10 300 python bench.py --scene 1 --width 1000 --height 1000 --spp 1000 --depth 30 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || { echo "bench c2 failed"; exit 1; }
timeout -k 10 300 python bench.py --scene 6 --width 4096 --height 4096 --spp 4096 --depth 20 --steps 1 --warmup 1 --no-cpu-baseline --no-reference-check > $O/c5.json 2> $O/c5.err || { echo "bench c5 failed"; exit 1; }
for c in c4 c3 c2 c5; do python -c "import json; d=json.load(open('$O/$c.json')); r=d['roofline']; print('$c', d['value'], d['kernel_ms_avg'], r.get('bound'), r.get('frac'), r.get('reason'), d['simd'])"; done
bash tools/gpu_rehearse_dist.sh $T/dist_c3 c3 || exit 1
bash tools/gpu_rehearse_dist.sh $T/dist_4k 4k || exit 1
echo final-done
