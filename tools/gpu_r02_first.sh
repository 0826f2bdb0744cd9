#!/bin/bash
# Round-2 first GPU check: the GPU test suite, the ceilings microbenchmark,
# the available PMC counters, and one default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-r02a}; mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 $R/build/ubench > $O/ubench.json 2> $O/ubench.err || { echo ubench failed; exit 1; }
cat $O/ubench.json
(cd /tmp && timeout -k 5 60 rocprofv3 -L > $O/counters.txt 2>&1); echo "counters rc=$?"
timeout -k 10 300 python $R/bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
