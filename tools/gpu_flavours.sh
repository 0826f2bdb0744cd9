#!/bin/bash
# GPU box: tools/flavour_check.py for the shipped library and each A/B variant named,
# then the bit-exact parity tests under the first variant.
# usage: bash tools/gpu_flavours.sh <tag> <variant>... [-- scene w h spp depth]
set -o pipefail
TAG=$1; shift
VARS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "$1" == "--" ] && shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
timeout -k 10 300 python tools/flavour_check.py "$@" >> $O/flavours.jsonl 2> $O/default.err || { echo "default failed"; tail -3 $O/default.err; exit 1; }
for v in "${VARS[@]}"; do
  ZRT_LIB=$R/abvar/$v/libzrt.so timeout -k 10 300 python tools/flavour_check.py "$@" >> $O/flavours.jsonl 2> $O/$v.err || { echo "$v failed"; tail -3 $O/$v.err; exit 1; }
done
cat $O/flavours.jsonl
if [ ${#VARS[@]} -gt 0 ]; then
  ZRT_LIB=$R/abvar/${VARS[0]}/libzrt.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "bit_exact" --timeout 300 --timeout-method thread > $O/parity_${VARS[0]}.log 2>&1; rc=$?
  tail -3 $O/parity_${VARS[0]}.log; exit $rc
fi
