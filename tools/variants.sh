#!/bin/bash
# Build kernel variants (compile-time knobs) into build/variants/<name>/libzrt.so.
# usage: bash tools/variants.sh name1="-DFOO=1" name2="-DBAR=2" ...
R=$(cd "$(dirname "$0")/.." && pwd)
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  mkdir -p $R/build/variants/$name
  make -s -j8 -C $R/zraytrace_amd/csrc OUT=$R/build/variants/$name/libzrt.so BUILD=$R/build/variants/$name/obj EXTRA="$flags" || exit 1
  echo "built $name ($flags)"
done
