"""Per-section cycle shares of the sampling loop (ZRT_PROFILE build; diagnostic).
usage: ZRT_LIB=abvar/prof/libzrt.so python tools/prof_sections.py [w h spp]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401  (shared HIP runtime)
import zraytrace_amd as z
w, h, spp = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (1024, 1024, 256)))
s = z.load_scene(2)
p = z.RenderParams(w, h, spp, 20)
ctx = z.RenderContext(s, p)
buf = torch.empty(ctx.tile_count(p) * 64 * 3, device="cuda")
ctx.render_tiles(s.camera, p, buf.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
c = ctx.debug_counters()
names = ["refill", "sample start", "traversal", "shading", "path end"]
tot = sum(c[16:21])
print("kernel ms", ctx.kernel_ms())
for n, v in zip(names, c[16:21]):
    print(f"{n:14s} {v / tot:6.1%}")
