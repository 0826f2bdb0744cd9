#!/bin/bash
# GPU box: the ceilings microbenchmarks with HIP-event times and the PMC counters
# bench.py's roofline divides by: tools/ubench.hip (generic VALU / load patterns)
# and tools/ubench_shapes.hip (the render kernel's own load shapes), prebuilt on
# the CPU as tools/ubench.bin and tools/ubench_shapes.bin:
#   hipcc --offload-arch=gfx950 -O3 -o tools/ubench.bin tools/ubench.hip
#   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_shapes.bin tools/ubench_shapes.hip
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${1:-ubench}; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 60 $R/tools/ubench.bin > $O/events.json 2> $O/events.err || { echo ubench failed; exit 1; }
timeout -k 10 120 $R/tools/ubench_shapes.bin > $O/events_shapes.json 2> $O/events_shapes.err || { echo ubench_shapes failed; exit 1; }
i=0
for grp in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $O/ub$i -o run -- $R/tools/ubench.bin > $O/ub$i.json 2> $O/ub$i.err || { echo "ubench pmc pass $i failed"; exit 1; }
done
i=0
for grp in "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_FLAT SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TD_TC_STALL_sum TA_FLAT_READ_LDS_WAVEFRONTS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/sh$i -o run -- $R/tools/ubench_shapes.bin > $O/sh$i.json 2> $O/sh$i.err || { echo "ubench_shapes pmc pass $i failed"; exit 1; }
done
python $R/tools/ubench_summary.py $O > $O/ubench.json && echo ubench-done
