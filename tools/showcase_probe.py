import sys, os, json
sys.path.insert(0, os.getcwd())
import numpy as np
import zraytrace_amd as z
s = z.load_scene(1)
img, st = z.render(s, s.camera, z.RenderParams(1000, 1000, 1000, 30))
q = np.trunc(np.clip(np.float32(255.999) * img, 0, 255))[::-1]
show = np.rint(z.read_png("assets/showcase-7-spheres.png")[::-1].astype(np.float64) * 255)
d = np.abs(q - show)
out = {"mean_gpu": q.reshape(-1, 3).mean(0).tolist(), "mean_show": show.reshape(-1, 3).mean(0).tolist(),
       "d_mean": d.mean(), "d_p99": float(np.percentile(d, 99)), "d_p999": float(np.percentile(d, 99.9)),
       "d_max": d.max(), "frac_le1": float((d <= 1).mean()), "frac_le2": float((d <= 2).mean()),
       "frac_le4": float((d <= 4).mean()), "rays": st["rays_processed"], "refl": st["reflections"], "bg": st["background_hits"]}
print(json.dumps(out))
