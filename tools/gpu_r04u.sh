#!/bin/bash
# GPU box, round 4: the lockstep loop's RNG state in LDS (lrng: 4 words per lane,
# 6 blocks/CU kept, spills 31 -> 23) against the shipped build, C4 and C3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04u; mkdir -p $O
cd $R
export TMPDIR=/tmp
export ZRT_DEBUG_LAUNCH=1
bash tools/ab.sh r04u/c4 2 default lrng -- --no-reference-check || exit 1
bash tools/ab.sh r04u/c3 2 default lrng -- --no-reference-check --scene 3 --width 1024 --height 1024 --spp 256 --depth 20 || exit 1
for f in $O/c4/*.json $O/c3/*.json; do python -c "import json; d=json.load(open('$f')); print('$f'.split('/')[-2:], d['frame_sha1'][:16])"; done
grep -h "zrt launch" $O/c4/*.1.err | sort -u | head -6
echo session-done
