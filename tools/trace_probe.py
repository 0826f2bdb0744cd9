"""Diagnose zrt_trace vs oracle mismatches (GPU box)."""
import sys, os, json
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np
import zraytrace_amd as z
from oracle import oracle_py as O
from zraytrace_amd import _ffi
import test_gpu_parity as T

scene_index = int(sys.argv[1]) if len(sys.argv) > 1 else 2
s = z.load_scene(scene_index)
v = s.view.contents
pr = T.prim_array(v)
tri = pr[pr["kind"] == _ffi.ZRT_PRIM_TRIANGLE]
verts = np.concatenate([tri["a"], tri["b"], tri["c"]]).reshape(-1, 3)
lo, hi = verts.min(0), verts.max(0)
rng = np.random.default_rng(scene_index)
n = 6000
o = rng.uniform(lo - (hi - lo), hi + (hi - lo), (n, 3)).astype(np.float32)
d = rng.normal(size=(n, 3)).astype(np.float32)
k = rng.integers(0, len(tri), 3000)
a = tri["a"][k]; b = tri["b"][k]; c = tri["c"][k]
targets = np.concatenate([a, (a + b) * np.float32(0.5), (a + b + c) / np.float32(3.0)]).astype(np.float32)
o2 = np.repeat(np.asarray([s.camera.origin.x, s.camera.origin.y, s.camera.origin.z], np.float32)[None],
               len(targets), 0) + rng.normal(scale=0.05, size=(len(targets), 3)).astype(np.float32)
kv = rng.integers(0, len(verts), 2000)
axis = np.eye(3, dtype=np.float32)[rng.integers(0, 3, 2000)] * rng.choice([-1, 1], (2000, 1)).astype(np.float32)
o3 = (verts[kv] - axis * np.float32(0.25)).astype(np.float32)
origins = np.concatenate([o, o2, o3]).astype(np.float32)
dirs = np.concatenate([d, targets - o2, axis]).astype(np.float32)
t_ref, p_ref = O.trace(s.view, True, origins, dirs)
t_list, p_list = O.trace(s.view, False, origins, dirs)
print("oracle bvh vs list mismatches:", int((p_ref != p_list).sum()))
for name, trav in (("fast", 0), ("reference", 1), ("binary", 2)):
    t, p = z.trace(s, z.RenderParams(1, 1, 1, 1, traversal=trav), origins, dirs)
    bad = np.nonzero((p != p_ref) | ~((t.view(np.uint32) == t_ref.view(np.uint32)) | (np.isinf(t) & np.isinf(t_ref))))[0]
    print(name, "mismatches", len(bad), "random:", int((bad < n).sum()), "vertex:", int(((bad >= n) & (bad < n + 3000)).sum()),
          "edge:", int(((bad >= n + 3000) & (bad < n + 6000)).sum()), "centroid:", int(((bad >= n + 6000) & (bad < n + 9000)).sum()), "axis:", int((bad >= n + 9000).sum()))
    for i in bad[:6]:
        print("  ray", int(i), "gpu", float(t[i]), int(p[i]), "ref", float(t_ref[i]), int(p_ref[i]), "list", float(t_list[i]), int(p_list[i]),
              "o", origins[i].tolist(), "d", dirs[i].tolist())
