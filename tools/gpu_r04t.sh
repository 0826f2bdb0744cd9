#!/bin/bash
# GPU box, round 4: the lockstep loop's RNG state and chunk sums in LDS with the
# LDS attenuation rows cut to 0 / 2 to make room (the 6-wave kernel's spills
# saturate TD on C4); launch geometry printed (ZRT_DEBUG_LAUNCH).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04t; mkdir -p $O
cd $R
export TMPDIR=/tmp
export ZRT_DEBUG_LAUNCH=1
bash tools/ab.sh r04t/c4 2 default lstr0 lstr2 -- --no-reference-check || exit 1
for f in $O/c4/*.json; do python -c "import json; d=json.load(open('$f')); print('$f'.split('/')[-1], d['frame_sha1'][:16])"; done
grep -h "zrt launch" $O/c4/*.1.err | sort -u | head -12
echo session-done
