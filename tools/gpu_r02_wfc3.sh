#!/bin/bash
# C3 / C4: lockstep loop (default for the 16-bit-stack scenes) vs the wavefront loop (ZRT_WF=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-r02wfc3}; mkdir -p $O; cd $R
for r in 1 2; do
for wf in 0 1; do
  ZRT_WF=$wf timeout -k 10 300 python bench.py --scene 3 --width 1024 --height 1024 --spp 256 --steps 5 --warmup 2 --no-cpu-baseline --no-reference-check > $O/c3_wf$wf.$r.json 2> $O/c3_wf$wf.$r.err || exit 1
  python -c "import json; d=json.load(open('$O/c3_wf$wf.$r.json')); print('C3 wf=$wf', d['value'], d['kernel_ms_avg'])"
done; done
