#!/bin/bash
# GPU box: config C5 substitute (scene 6) bench line + rocprofv3 kernel stats and
# PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) of the same workload.
# usage: bash tools/gpu_c5prof.sh <tag> [spp]
set -o pipefail
TAG=${1:-c5prof}; SPP=${2:-4096}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
A="--scene 6 --width 4096 --height 4096 --spp $SPP --depth 20"
timeout -k 10 600 python $R/bench.py $A > $O/c5.json 2> $O/c5.err || { echo "c5 bench failed"; tail -3 $O/c5.err; exit 1; }
tail -1 $O/c5.json | cut -c1-200
P="$A --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python $R/bench.py $P > $O/trace.json 2> $O/trace.err || { echo "trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python $R/bench.py $P > $O/pmc_fetch.json 2> $O/pmc_fetch.err || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python $R/bench.py $P > $O/pmc_write.json 2> $O/pmc_write.err || { echo "pmc write failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/pmc_sq -o run -- python $R/bench.py $P > $O/pmc_sq.json 2> $O/pmc_sq.err || { echo "pmc sq failed"; exit 1; }
python $R/tools/pmc_summary.py $O $O/pmc_traffic.json && echo c5prof-done
