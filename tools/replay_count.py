"""Order-hazard replays per ray (ZRT_FLAG_STATS) for a few scenes (GPU box)."""
import sys, os
sys.path.insert(0, os.getcwd())
import zraytrace_amd as z
for idx, w, spp in ((2, 2048, 16), (3, 1024, 16), (0, 512, 16), (4, 512, 16)):
    s = z.load_scene(idx)
    for trav, name in ((z.ZRT_TRAVERSAL_FAST, "fast"), (z.ZRT_TRAVERSAL_BINARY, "binary")):
        _, st = z.render(s, s.camera, z.RenderParams(w, w, spp, 20, traversal=trav, flags=z.ZRT_FLAG_STATS))
        print(idx, name, st["rays_processed"], st["order_replays"], st["order_replays"] / st["rays_processed"], flush=True)
