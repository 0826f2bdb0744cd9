#!/bin/bash
# Round 2: scanline/CLI GPU tests, then SIMD efficiency (STATS counters) per config.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-r02eff}; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "scanline or cli" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/simd_eff.py 2:2048:2048:16 3:1024:1024:16 1:1000:1000:16 6:4096:4096:4 > $O/eff.jsonl 2> $O/eff.err || { tail -5 $O/eff.err; exit 1; }
cat $O/eff.jsonl
