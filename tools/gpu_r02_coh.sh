#!/bin/bash
# Round 2: coherence of the FAST loop's fetches (STATS counters) per config.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-r02coh}; mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/simd_eff.py 2:2048:2048:16 3:1024:1024:16 6:4096:4096:4 > $O/eff.jsonl 2> $O/eff.err || { tail -5 $O/eff.err; exit 1; }
cat $O/eff.jsonl
ZRT_WF=0 timeout -k 10 300 python -u tools/simd_eff.py 6:4096:4096:4 > $O/eff_c5_lock.jsonl 2>> $O/eff.err || exit 1
cat $O/eff_c5_lock.jsonl
