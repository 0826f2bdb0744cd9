#!/bin/bash
# GPU box: full bench + rocprofv3 kernel trace/stats of the same command +
# separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ instruction counters) of a one-launch run.
# Usage: bash tools/gpu_profile.sh <tag>
set -o pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 python $R/bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python $R/bench.py --no-cpu-baseline > $OUT/bench_traced.json 2> $OUT/trace.err || { echo "trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_write.json 2> $OUT/pmc_write.err || { echo "pmc write failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES --output-format csv -d $OUT/pmc_sq -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err || { echo "pmc sq failed"; exit 1; }
python $R/tools/pmc_summary.py $OUT $OUT/pmc_traffic.json && echo profile-done
