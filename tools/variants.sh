#!/bin/bash
# Build kernel variants (compile-time knobs) into abvar/<name>/libzrt.so for an
# A/B session (tools/ab.sh, tools/gpu_ab2.sh).  abvar/ is git-ignored and NOT
# gpurun-ignored, so the variants travel to the GPU box only while they exist:
# many are deliberately inexact (A/B probes), so remove them after the session
#   bash tools/variants.sh --clean
# usage: bash tools/variants.sh name1="-DFOO=1" name2="-DBAR=2" ...
R=$(cd "$(dirname "$0")/.." && pwd)
if [ "$1" == "--clean" ]; then rm -rf "$R/abvar"; echo "removed abvar/"; exit 0; fi
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  mkdir -p $R/abvar/$name
  make -s -j8 -C $R/zraytrace_amd/csrc OUT=$R/abvar/$name/libzrt.so BUILD=$R/build/variants/$name/obj CLI=$R/abvar/$name/zrt-raytrace EXTRA="$flags" || exit 1
  echo "built $name ($flags)"
done
