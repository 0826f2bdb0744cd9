"""How far the reference's closest hits lie outside their own primitive's box, on the
grazing rays of tests/grazing_rays.py, against the FAST culls' margins (DESIGN.md §3
"Grazing rays").  CPU only: the oracle's trace (the reference's BVH traversal) gives
each ray's hit; the hit point o + t*unit(d) is compared with the primitive's box
(triangle: vertex min/max; sphere: center -+ r), axis by axis.

A box FAST culls has entry > exit * rel + slack (render.hip ray_slack: rel = 1 +
2^-16 + 2^-18 M, slack = 2^-18 x the triangles' largest |coordinate| x M, M =
max_k |1/d_k|); a hit outside its box by e_k on axis k lies e_k * |1/d_k| outside the
box's t interval.  Printed: the largest spatial excess relative to max(scene extent,
|o|), and the largest t-space excess as a fraction of half the cull margin, in the
slack form (reference boxes; triangles and spheres apart: a sphere's hit point is
on the ray, its excess is its error in t) and in the local form (2^-19 x the box's own largest
|coordinate| x |1/d_k| + t (2^-16 + 2^-18 M) / 2: grown inner boxes, loose_slot) - below
1 means every hit of these rays would survive the cull.

usage: python tools/grazing_excess.py [scene ...]   (default 0 2 3 4)
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import zraytrace_amd as z  # noqa: E402
from oracle import oracle_py as O  # noqa: E402
import grazing_rays as G  # noqa: E402
from test_gpu_parity import prim_array  # noqa: E402


def main():
    scenes = [int(s) for s in sys.argv[1:]] or [0, 2, 3, 4]
    for w in scenes:
        keep = z.load_scene(w)
        v = keep.view
        pr = prim_array(v.contents if hasattr(v, "contents") else v)
        mins, maxs, left, _, _ = O.bvh_build(v)
        o, d = G.grazing_rays(pr, mins, maxs, left, n=6000, seed=7, span=float(np.max(maxs[0] - mins[0])))
        t, p = O.trace(v, True, o, d)
        tri = pr["kind"] == 1
        V = np.stack([pr["a"], pr["b"], pr["c"]], 1).astype(np.float64)
        r = np.abs(pr["radius"]).astype(np.float64)[:, None]
        c = pr["center"].astype(np.float64)
        lo = np.where(tri[:, None], V.min(1), c - r)
        hi = np.where(tri[:, None], V.max(1), c + r)
        extent = max(np.abs(lo).max(), np.abs(hi).max())
        h = p >= 0
        u = d[h].astype(np.float64)
        u /= np.linalg.norm(u, axis=1, keepdims=True)
        x = o[h].astype(np.float64) + t[h, None].astype(np.float64) * u
        e = np.maximum(lo[p[h]] - x, 0) + np.maximum(x - hi[p[h]], 0)
        scale = np.maximum(extent, np.abs(o[h]).max(1))
        with np.errstate(divide="ignore"):
            inv = np.abs(1.0 / u)
        m = inv.max(1)
        et = np.nan_to_num(e * inv, nan=0.0, posinf=0.0).max(1)
        ctri = max(np.abs(V[tri]).max(), 1e-30) if tri.any() else 1e-30
        half = 2.0 ** -19 * ctri * m + t[h] * (2.0 ** -16 + 2.0 ** -18 * m) / 2
        # the local form (inner wide boxes, loose_slot): per axis 2^-19 x the box's own
        # largest |coordinate| (here the primitive's, the smallest box holding it)
        # x |1/d_k|, plus t x (2^-16 + 2^-18 M) / 2
        cp = np.maximum(np.abs(lo[p[h]]).max(1), np.abs(hi[p[h]]).max(1))
        loc = np.nan_to_num(2.0 ** -19 * cp[:, None] * inv, nan=np.inf) + (t[h] * (2.0 ** -16 + 2.0 ** -18 * m) / 2)[:, None]
        with np.errstate(invalid="ignore"):
            rl = np.nan_to_num(e * inv / loc, nan=0.0).max(1)
        th = tri[p[h]]
        rs = et / half
        print(f"scene {w}: {int(h.sum())} hits, extent {extent:.4g}, triangles' {ctri:.4g}; spatial excess / "
              f"max(extent, |o|) max {(e.max(1) / scale).max():.3g}; t-space excess / half margin max: "
              f"slack form triangles {rs[th].max() if th.any() else 0:.3g} spheres "
              f"{rs[~th].max() if (~th).any() else 0:.3g}, local form {rl.max():.3g}")


if __name__ == "__main__":
    main()
