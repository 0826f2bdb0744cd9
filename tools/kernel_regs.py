"""Register / spill / LDS use of the render kernels from device assembly.

usage: python tools/kernel_regs.py <render.s>   (hipcc ... --cuda-device-only -S)
"""
import re
import sys

s = open(sys.argv[1]).read()
meta = s[s.index("amdhsa.kernels:"):]
for blk in meta.split("  - .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if "render_kernel" not in name and "probe" not in name and "trace_kernel" not in name:
        continue
    g = lambda k: (re.search(r"\.%s:\s+(\d+)" % k, blk) or [None, None])[1]
    print(f"{name[:70]:70s} vgpr {g('vgpr_count')} spill {g('vgpr_spill_count')} sgpr {g('sgpr_count')} "
          f"sspill {g('sgpr_spill_count')} private {g('private_segment_fixed_size')}")
