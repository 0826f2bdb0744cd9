#!/bin/bash
# GPU box, round 4 shipped build: rocprofv3 --kernel-trace --stats of the driver's
# exact default bench command (C4 with the CPU baseline and the REFERENCE frame).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04final/rocprof_default; mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/bench.py > $O/bench.json 2> $O/bench.err || { echo "traced bench failed"; tail -5 $O/bench.err; exit 1; }
tail -1 $O/bench.json
find $O -name '*.csv' ! -name '*kernel_stats.csv' -size +1M -exec gzip -9 {} \;
echo session-done
