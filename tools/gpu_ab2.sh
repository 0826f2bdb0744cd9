#!/bin/bash
# GPU box: interleaved A/B of library builds and/or environment knobs.
# usage: bash tools/gpu_ab2.sh <tag> <rounds> <spec>... [-- bench args]
#   spec = name=<variant or default>[:VAR=val[,VAR=val...]]
#   e.g.  bash tools/gpu_ab2.sh ab 2 new=default old=nolds noatt=default:ZRT_ATT_LDS_ROWS=0 -- --steps 3
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
SPECS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do SPECS+=("$1"); shift; done
[ "$1" == "--" ] && shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for spec in "${SPECS[@]}"; do
    name=${spec%%=*}; rest=${spec#*=}; v=${rest%%:*}; envs=""; [ "$rest" != "$v" ] && envs=${rest#*:}
    if [ "$v" == "default" ]; then LIB=$R/zraytrace_amd/libzrt.so; else LIB=$R/abvar/$v/libzrt.so; fi
    env ZRT_LIB=$LIB ${envs//,/ } timeout -k 10 300 python $R/bench.py --no-cpu-baseline --no-reference-check "$@" > $OUT/$name.$r.json 2> $OUT/$name.$r.err || { echo "variant $name failed"; tail -5 $OUT/$name.$r.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/$name.$r.json')); print('$name', $r, d['value'], 'Mrays/s', d['kernel_ms_avg'], 'ms', d['frame_sha1'][:12])"
  done
done
