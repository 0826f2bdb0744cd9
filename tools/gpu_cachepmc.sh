#!/bin/bash
# GPU box: L1 (TCP) / TLB (UTCL1) / L2 (TCC) counters of the render kernel, one
# rocprofv3 --pmc pass per counter group, for a given bench workload.
# usage: bash tools/gpu_cachepmc.sh <tag> <bench args...>
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
P="$* --steps 1 --warmup 0 --no-cpu-baseline"
i=0
for grp in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
           "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python $R/bench.py $P > $O/p$i.json 2> $O/p$i.err || { echo "pass $i failed"; tail -3 $O/p$i.err; exit 1; }
done
echo cachepmc-done
