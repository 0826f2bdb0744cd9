#!/bin/bash
# A/B build variants on the GPU box: interleaved rounds of bench.py per variant.
# usage: bash tools/ab.sh <tag> <rounds> <variant>[@chunk]... [-- bench args]
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
VARS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "$1" == "--" ] && shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for spec in "${VARS[@]}"; do
    v=${spec%%@*}; EXTRA_ARGS=(); [ "$spec" != "$v" ] && EXTRA_ARGS=(--chunk ${spec#*@})
    if [ "$v" == "default" ]; then LIB=$R/zraytrace_amd/libzrt.so; else LIB=$R/abvar/$v/libzrt.so; fi
    ZRT_LIB=$LIB timeout -k 10 300 python $R/bench.py --no-cpu-baseline "$@" "${EXTRA_ARGS[@]}" > $OUT/$spec.$r.json 2> $OUT/$spec.$r.err || { echo "variant $v failed"; tail -5 $OUT/$spec.$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$OUT/$spec.$r.json')); print('$spec', $r, d['build_id'], d['value'], 'Mrays/s', d['kernel_ms_avg'], 'ms', d['roofline']['algorithmic']['per_ray'])"
  done
done
# every variant must have run its own library (a library rebuilt in place between
# builds - tests/conftest.py rebuilds a stale in-tree one - would make two the same)
python - "$OUT" <<'PYEOF' || exit 1
import glob, json, os, sys
ids = {}
for f in glob.glob(os.path.join(sys.argv[1], "*.json")):
    v = os.path.basename(f).rsplit(".", 2)[0].split("@")[0]  # (v@chunk: one library, several chunks)
    ids.setdefault(json.load(open(f))["build_id"], set()).add(v)
dup = [sorted(vs) for vs in ids.values() if len(vs) > 1]
if dup:
    sys.exit(f"A/B invalid: variants {dup} ran the same library")
PYEOF
