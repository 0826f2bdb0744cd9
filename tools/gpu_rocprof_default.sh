#!/bin/bash
# GPU box: rocprofv3 --kernel-trace --stats of the driver's default bench command
# (python bench.py, no arguments): the per-kernel summary committed under profiles/.
# usage: bash tools/gpu_rocprof_default.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$1/rocprof_default; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python $R/bench.py > $O/bench.json 2> $O/bench.err || { echo "rocprof default failed"; tail -3 $O/bench.err; exit 1; }
find $O -name '*.csv' ! -name '*kernel_stats.csv' -size +1M -exec gzip -9 {} \;
grep -E "render_kernel|probe|finalize" $O/run_kernel_stats.csv | cut -c1-150
