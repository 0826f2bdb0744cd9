#!/bin/bash
# GPU box: the ceilings microbenchmark (tools/ubench.hip, prebuilt as abvar/ubench)
# with HIP-event times and the PMC counters bench.py's roofline divides by.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-ubench}; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 $R/abvar/ubench > $O/events.json 2> $O/events.err || { echo ubench failed; exit 1; }
i=0
for grp in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $O/ub$i -o run -- $R/abvar/ubench > $O/ub$i.json 2> $O/ub$i.err || { echo "ubench pmc pass $i failed"; exit 1; }
done
python $R/tools/ubench_summary.py $O > $O/ubench.json && cat $O/ubench.json
