#!/bin/bash
# GPU box, round 4: room for the lockstep lane state in LDS by reading the top
# wide nodes from global memory (ZRT_LDS_TOP=0): notop alone, and with the RNG
# state + chunk sums in LDS (lstnotop), against the shipped build on C4 and C3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04x; mkdir -p $O
cd $R
export TMPDIR=/tmp
export ZRT_DEBUG_LAUNCH=1
bash tools/ab.sh r04x/c4 2 default notop lstnotop -- --no-reference-check || exit 1
bash tools/ab.sh r04x/c3 1 default notop lstnotop -- --no-reference-check --scene 3 --width 1024 --height 1024 --spp 256 --depth 20 || exit 1
for f in $O/c4/*.json $O/c3/*.json; do python -c "import json; d=json.load(open('$f')); print('$f'.split('/')[-2:], d['frame_sha1'][:16])"; done
grep -h "zrt launch" $O/c4/*.1.err | sort -u | head -6
echo session-done
