"""One timed FAST render launch (no STATS flavour), for profilers that sample the
kernel (tools/gpu_pcsample.sh).  usage: python tools/render_once.py [scene w h spp depth]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import zraytrace_amd as z  # noqa: E402

a = [int(x) for x in sys.argv[1:]]
scene_i = a[0] if a else 2
w, h, spp, depth = a[1:5] if len(a) >= 5 else (1024, 1024, 64, 20)
s = z.load_scene(scene_i)
_, st = z.render(s, s.camera, z.RenderParams(w, h, spp, depth))
print(json.dumps({"build_id": z.build_id(), "config": [scene_i, w, h, spp, depth], "render_ms": round(st["render_ms"], 2)}))
