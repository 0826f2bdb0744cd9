"""Distribution of wave start/end times of one launch (ZRT_PROFILE build; diagnostic).
usage: ZRT_LIB=build/variants/prof/libzrt.so python tools/wave_times.py [w h spp] [noschedule]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch  # noqa: F401
import zraytrace_amd as z

w, h, spp = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (2048, 2048, 128)))
flags = z.ZRT_FLAG_NO_SCHEDULE if "noschedule" in sys.argv else 0
s = z.load_scene(2)
p = z.RenderParams(w, h, spp, 20, flags=flags)
ctx = z.RenderContext(s, p)
buf = torch.empty(ctx.tile_count(p) * 64 * 3, device="cuda")
for _ in range(2):
    ctx.render_tiles(s.camera, p, buf.data_ptr(), torch.cuda.current_stream().cuda_stream)
t = ctx.debug_wave_times().astype(np.int64)
t0 = t[:, 0].min()
start, end = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0  # microseconds
q = lambda a, f: np.quantile(a, f)
print(f"{w}x{h}@{spp} {'no schedule' if flags else 'scheduled'}: kernel {ctx.kernel_ms():.2f} ms, waves {len(t)}; "
      f"start max {start.max():.0f} us; end min {end.min():.0f} p10 {q(end, .1):.0f} p50 {q(end, .5):.0f} "
      f"p90 {q(end, .9):.0f} p99 {q(end, .99):.0f} max {end.max():.0f} us; mean busy {np.mean(end - start):.0f} us")
