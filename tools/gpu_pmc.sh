#!/bin/bash
# GPU box: rocprofv3 evidence for one bench.py workload - a --kernel-trace
# --stats pass of the bench command, then one --pmc pass per counter group
# (each pass its own run: the hardware limits per block, MI355X_MICROARCH.md)
# of a one-step run.  (A counter appears in one pass only: pmc_summary.py adds
# the passes' counts.)  pmc_summary.py turns them into the entry bench.py's
# roofline reads (tools/make_latest_pmc.py merges it into profiles/latest_pmc.json).
# usage: bash tools/gpu_pmc.sh <tag> [bench args...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B="$R/bench.py $* --no-cpu-baseline --no-reference-check"
echo "bench args: $*" > $O/args.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $B > $O/bench_traced.json 2> $O/trace.err || { echo "trace pass failed"; tail -3 $O/trace.err; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
           "TD_TC_STALL_sum TD_LOAD_WAVEFRONT_sum TA_FLAT_READ_WAVEFRONTS_sum TA_FLAT_READ_LDS_WAVEFRONTS_sum SQ_INSTS_FLAT SQ_INSTS_SMEM" \
           "TD_STORE_WAVEFRONT_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $grp --output-format csv -d $O/pmc$i -o run -- python $B --steps 1 --warmup 0 > $O/pmc$i.json 2> $O/pmc$i.err || { echo "pmc pass $i ($grp) failed"; tail -3 $O/pmc$i.err; exit 1; }
done
python $R/tools/pmc_summary.py $O > $O/entry.json || exit 1
# gpurun copies back at most 64 MiB: keep the summaries, compress the raw CSVs
# (the BVH build's radix-sort launches make a million-triangle scene's large)
find $O -name '*.csv' ! -name '*kernel_stats.csv' -size +1M -exec gzip -9 {} \;
find $O -name '*.csv.gz' -size +8M -delete
echo pmc-done
