"""Kernel time of each rank's share of a frame, rendered one rank at a time on
one GPU: how much of the N-GPU step is tail (diagnostic).
usage: python tools/tail_probe.py [world] [scene w h spp depth]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401  (shared HIP runtime)
import zraytrace_amd as z
from zraytrace_amd.dist import tile_counts

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
chunk = int(os.environ.get("ZRT_CHUNK", "0"))
scene, w, h, spp, depth = (int(x) for x in (sys.argv[2:7] if len(sys.argv) > 6 else (2, 2048, 2048, 1024, 20)))
s = z.load_scene(scene)
stream = torch.cuda.current_stream().cuda_stream
full = z.RenderParams(w, h, spp, depth, sample_chunk=chunk)
ctx = z.RenderContext(s, full)
buf = torch.empty(ctx.tile_count(full) * 64 * 3, device="cuda")
ctx.render_tiles(s.camera, full, buf.data_ptr(), stream)
ctx.render_tiles(s.camera, full, buf.data_ptr(), stream)
t1 = ctx.kernel_ms()
per, sched, total = [], [], []
for r in range(world):
    p = z.RenderParams(w, h, spp, depth, rank=r, world_size=world, sample_chunk=chunk)
    ctx.render_tiles(s.camera, p, buf.data_ptr(), stream)
    per.append(ctx.kernel_ms())
    st = ctx.stats()
    sched.append(st["schedule_ms"])
    total.append(st["render_ms"])
print(f"1 GPU: {t1:.1f} ms; {world} ranks: {', '.join(f'{x:.1f}' for x in per)} ms; "
      f"ideal {t1 / world:.1f}, max {max(per):.1f} -> kernel efficiency {t1 / world / max(per):.3f}; "
      f"tiles {tile_counts(z.RenderParams(w, h, spp, depth, world_size=world))[:2]}; "
      f"schedule ms {max(sched):.2f}; max render_ms (probe + sort + kernel) {max(total):.2f}")
if len(sys.argv) > 7:
    import numpy as np
    p = z.RenderParams(w, h, spp, depth, rank=world - 1, world_size=world)
    ctx.render_tiles(s.camera, p, buf.data_ptr(), stream)
    costs, order = ctx.debug_schedule()
    c = np.sort(costs.astype(np.float64))[::-1]
    n_groups = (spp + 63) // 64
    waves = 6144
    # probe iterations cover 4 samples; a unit covers 64 (one chunk)
    unit = c * 16
    print(f"probe costs (iterations / 4 spp): mean {c.mean():.1f}, p50 {np.median(c):.0f}, p99 {c[len(c) // 100]:.0f}, "
          f"max {c[0]:.0f}; top {c[:6].astype(int).tolist()}; per-wave unit budget {unit.sum() * n_groups / waves:.0f} "
          f"vs largest unit {unit[0]:.0f} iterations")
    sys.exit(0)
rays = []
for r in range(world):
    p = z.RenderParams(w, h, spp, depth, rank=r, world_size=world)
    ctx.render_tiles(s.camera, p, buf.data_ptr(), stream)
    rays.append(ctx.stats()["rays_processed"])
print("rays per rank (M):", [round(x / 1e6, 1) for x in rays], "time per Grays:",
      [round(t / (x / 1e9), 2) for t, x in zip(per, rays)])
for div in (2, 4, 8):  # smaller whole frames: is a short kernel itself inefficient?
    ws = int(round(w / div ** 0.5 / 8)) * 8
    p = z.RenderParams(ws, ws, spp, depth)
    c2 = z.RenderContext(s, p)
    b2 = torch.empty(c2.tile_count(p) * 64 * 3, device="cuda")
    c2.render_tiles(s.camera, p, b2.data_ptr(), stream)
    c2.render_tiles(s.camera, p, b2.data_ptr(), stream)
    st = c2.stats()
    print(f"frame {ws}^2: {c2.kernel_ms():.1f} ms, {st['rays_processed'] / c2.kernel_ms() / 1e6:.1f} Grays/s")
    c2.close()
