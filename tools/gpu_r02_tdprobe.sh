#!/bin/bash
# Cache / TD counters of the C4 render launch for two library builds in one
# session (is a change of TCP accesses / TD busy between PMC entries real?).
# usage: bash tools/gpu_r02_tdprobe.sh <tag> <variant>...   (default = in-tree libzrt.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; T=$1; shift; O=$R/gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  if [ "$v" == "default" ]; then LIB=$R/zraytrace_amd/libzrt.so; else LIB=$R/build/variants/$v/libzrt.so; fi
  ZRT_LIB=$LIB timeout -s KILL 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d $O/$v -o run -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-reference-check > $O/$v.json 2> $O/$v.err || { echo "pass $v failed"; tail -3 $O/$v.err; exit 1; }
  python - "$O/$v/run_counter_collection.csv" "$v" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
for row in csv.DictReader(open(sys.argv[1])):
    k = row.get("Kernel_Name", "")
    if "render_kernel<3, 0, false" in k:
        acc[row["Counter_Name"]] += float(row["Counter_Value"])
print(sys.argv[2], dict(acc))
PY
done
