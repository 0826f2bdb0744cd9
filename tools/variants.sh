#!/bin/bash
# Build kernel variants (compile-time knobs) into abvar/<name>/libzrt.so for an
# A/B session (tools/ab.sh, tools/gpu_ab2.sh).  abvar/ is git-ignored, and
# gpurun-ignored (./abvar in .gpurunignore) except while variants exist: building
# them lifts that line so they travel to the GPU box for the A/B session; --clean
# removes them (many are deliberately inexact A/B probes) and restores the line
#   bash tools/variants.sh --clean
# usage: bash tools/variants.sh name1="-DFOO=1" name2="-DBAR=2" ...
R=$(cd "$(dirname "$0")/.." && pwd)
if [ "$1" == "--clean" ]; then
  rm -rf "$R/abvar"; grep -qx './abvar' $R/.gpurunignore || echo './abvar' >> $R/.gpurunignore
  echo "removed abvar/ (gpurun-ignored again)"; exit 0
fi
sed -i '/^\.\/abvar$/d' $R/.gpurunignore
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  mkdir -p $R/abvar/$name
  make -s -j8 -C $R/zraytrace_amd/csrc OUT=$R/abvar/$name/libzrt.so BUILD=$R/build/variants/$name/obj CLI=$R/abvar/$name/zrt-raytrace EXTRA="$flags" || exit 1
  echo "built $name ($flags)"
done
