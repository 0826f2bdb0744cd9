"""GPU box: how far the hits the reference computes lie outside their own leaf's
box (DESIGN.md §3 "Exactness", assumption A): one REFERENCE-traversal launch of
the STATS flavour per scene (zrt_stats.box_excess_*), at the bench's resolution
with a few samples per pixel.

usage: python tools/box_excess.py [spp]   -> one JSON line per scene
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import zraytrace_amd as z  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 4
for idx, (w, h, depth) in ((2, (2048, 2048, 20)), (3, (1024, 1024, 20)), (0, (1024, 1024, 20)),
                           (4, (1024, 1024, 20))):
    s = z.load_scene(idx)
    p = z.RenderParams(w, h, spp, depth, traversal=z.ZRT_TRAVERSAL_REFERENCE, flags=z.ZRT_FLAG_STATS)
    _, st = z.render(s, s.camera, p)
    print(json.dumps({"scene": idx, "width": w, "height": h, "spp": spp, "rays": st["rays_processed"],
                      "prim_tests": st["prim_tests"], "box_excess_max_triangle": st["box_excess_max_triangle"],
                      "box_excess_max_sphere": st["box_excess_max_sphere"],
                      "box_excess_hits_over_2^-14": st["box_excess_hits"], "render_ms": round(st["render_ms"], 1)}),
          flush=True)
