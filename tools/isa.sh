#!/bin/bash
# Device assembly of one render kernel, for register / spill / instruction probes
# (seconds, not the full library's minutes).  The library it would link is never
# built: the other kernels are not instantiated (render.hip ZRT_ISA_KERNEL).
# usage: bash tools/isa.sh <out.s> ["MODE, PRNG, STATS, StackT"] [extra hipcc flags...]
#   default kernel: the C4 lockstep FAST kernel "3, 0, false, uint16_t"
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$1; K=${2:-"3, 0, false, uint16_t"}; shift; [ $# -gt 0 ] && shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wno-unused-function \
  --offload-arch=gfx950 -munsafe-fp-atomics -fno-slp-vectorize --cuda-device-only -S \
  "-DZRT_ISA_KERNEL=$K" "$@" -o $OUT $R/zraytrace_amd/csrc/render.hip 2>&1 | grep -v 'unused-command-line' 
python $R/tools/kernel_regs.py $OUT
