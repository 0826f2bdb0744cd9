#!/bin/bash
# GPU box, round 4: the whole GPU suite on the guard build, then bench lines of C4, C3, C2, C5.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r04g; mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu_session.sh r04g/s --no-tests bench:c3 bench:c2 bench:c5 || exit 1
echo session-done
