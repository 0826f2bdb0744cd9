#!/bin/bash
# GPU box, round 4 final build (3b7c974e): the full GPU suite, smoke, an A/B of the
# lockstep loop's lane state in LDS (abvar/lst) on C4 and C3 with frame hashes,
# the bench lines of C4 (CPU baseline + REFERENCE-traversal frame), C3, C2, C5,
# and the gloo rehearsals of C3 and the tiled 4K frame.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=r04final; O=$R/gpurun_out/$T; mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
bash tools/ab.sh $T/ab_lst_c4 2 default lst -- --no-reference-check || exit 1
bash tools/ab.sh $T/ab_lst_c3 1 default lst -- --no-reference-check --scene 3 --width 1024 --height 1024 --spp 256 --depth 20 || exit 1
for f in $O/ab_lst_c4/*.json $O/ab_lst_c3/*.json; do python -c "import json; d=json.load(open('$f')); print('$f'.split('/')[-2:], d['frame_sha1'][:16])"; done
timeout -k 10 600 python bench.py > $O/c4.json 2> $O/c4.err || { echo "bench c4 failed"; tail -5 $O/c4.err; exit 1; }
timeout -k 10 300 python bench.py --scene 3 --width 1024 --height 1024 --spp 256 --depth 20 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { echo "bench c3 failed"; exit 1; }
timeout -k 10 300 python bench.py --scene 1 --width 1000 --height 1000 --spp 1000 --depth 30 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || { echo "bench c2 failed"; exit 1; }
timeout -k 10 300 python bench.py --scene 6 --width 4096 --height 4096 --spp 4096 --depth 20 --steps 1 --warmup 1 --no-cpu-baseline --no-reference-check > $O/c5.json 2> $O/c5.err || { echo "bench c5 failed"; exit 1; }
for c in c4 c3 c2 c5; do python -c "import json; d=json.load(open('$O/$c.json')); r=d['roofline']; print('$c', d['value'], d['kernel_ms_avg'], r.get('bound'), r.get('frac'), d['simd'])"; done
bash tools/gpu_rehearse_dist.sh $T/dist_4k 4k || exit 1
bash tools/gpu_rehearse_dist.sh $T/dist_c3 c3 || exit 1
echo final-done
