#!/bin/bash
# GPU box: interleaved A/B of environment settings on the default build.
# usage: bash tools/gpu_env_ab.sh <tag> <rounds> "<NAME=VAL ...>" "<NAME=VAL ...>" ... -- <bench args>
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
ENVS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do ENVS+=("$1"); shift; done
[ "$1" == "--" ] && shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  i=0
  for e in "${ENVS[@]}"; do
    i=$((i + 1))
    env $e timeout -k 10 300 python $R/bench.py --no-cpu-baseline "$@" > $OUT/e$i.$r.json 2> $OUT/e$i.$r.err || { echo "env '$e' failed"; tail -5 $OUT/e$i.$r.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/e$i.$r.json')); print('$e', $r, d['value'], 'Mrays/s', d['kernel_ms_avg'], 'ms')"
  done
done
