#!/bin/bash
# GPU box: the round's final evidence for the shipped library - the C5 PMC passes
# (tools/gpu_pmc.sh), bench lines of C4 (full: CPU baseline + REFERENCE-traversal
# frame), C3 and C2 (their PMC entries are in profiles/latest_pmc.json, so the
# lines carry the roofline), the N-rank rehearsal over gloo, and a runtime A/B.
# usage: bash tools/gpu_final.sh <tag> [--pmc-c5] [ab-args for tools/gpu_ab2.sh ...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O
(cd $R && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1) || { echo "smoke failed"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
if [ "$1" == "--pmc-c5" ]; then
  shift
  bash $R/tools/gpu_pmc.sh $TAG/pmc_c5 --scene 6 --width 4096 --height 4096 --spp 4096 --depth 20 --steps 1 --warmup 0 || exit 1
fi
(cd $R && timeout -k 10 600 python bench.py > $O/c4.json 2> $O/c4.err) || { echo "bench c4 failed"; tail -5 $O/c4.err; exit 1; }
(cd $R && timeout -k 10 300 python bench.py --scene 3 --width 1024 --height 1024 --spp 256 --depth 20 --no-cpu-baseline > $O/c3.json 2> $O/c3.err) || { echo "bench c3 failed"; exit 1; }
(cd $R && timeout -k 10 300 python bench.py --scene 1 --width 1000 --height 1000 --spp 1000 --depth 30 --no-cpu-baseline > $O/c2.json 2> $O/c2.err) || { echo "bench c2 failed"; exit 1; }
for c in c4 c3 c2; do python -c "import json; d=json.load(open('$O/$c.json')); r=d['roofline']; print('$c', d['value'], d['kernel_ms_avg'], r.get('bound'), r.get('frac'), r.get('reason'), d['simd'])"; done
bash $R/tools/gpu_rehearse_dist.sh $TAG/dist || exit 1
[ $# -gt 0 ] && { bash $R/tools/gpu_ab2.sh "$@" || exit 1; }
echo final-done
