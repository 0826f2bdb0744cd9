"""Grazing-triangle rays: the corner of FAST's exactness argument that rests on
measurement (DESIGN.md §3 "Triangles: what the margins cover").

triangle.zig:48-70 accepts a hit when the ROUNDED barycentrics pass, so the
exact point where the ray crosses the triangle's plane may lie outside the
triangle - and outside its reference leaf's box - by up to about
K u |ao| |e1| |e2| / det (u = 2^-24; K ~ 2.6 measured, tools/tri_reach.py).  For
rays nearly parallel to the plane (det small against |e1| |e2|) that reach
exceeds the margins of FAST's narrowed box test, which could then cull a leaf
whose triangle the reference hits.

The rays here are built to land exactly there, on the scene's own triangles:
* a triangle T of reference leaf L and a vertex v of T lying on a face of L's
  box (axis k, side s: v_k is L's min or max on k);
* a point P = v + g w in T's plane, w the in-plane direction of s e_k: P lies
  outside T and outside L's box on axis k by about g |w_k|;
* a direction d at incidence det = -d . n in [1e-6, 1e-3] (n = e1 x e2 as the
  reference stores it; det >= 1e-6 is the reference's own acceptance bound),
  running through P from a random in-plane heading;
* g log-uniform over 0.02 .. 4 x the measured reach at that det, so a good
  share of the rays is accepted by the rounded test although it misses T.
The triangles are drawn with weight |e1| |e2| (the large ones reach farthest).

Test infrastructure (tests/test_gpu_parity.py, tools/grazing_tris_probe.py,
tests/golden/make_grazing_golden.py): every traversal must equal oracle_trace
bit for bit on these rays.
"""
import numpy as np

U = 2.0 ** -24


def leaf_candidates(prims, mins, maxs, left, right):
    """(tri index, vertex 0..2, axis, side +-1, leaf) for every triangle vertex
    lying on a face of its reference leaf's box (prims: zrt_prim structured
    array; mins/maxs/left/right: the reference BVH, children < 0 = -(prim) - 1)."""
    leaves = np.nonzero(left < 0)[0]
    pa, pb = -left[leaves] - 1, -right[leaves] - 1
    out = []
    for pr_col in (pa, pb):
        for vi, f in enumerate(("a", "b", "c")):
            tri = prims["kind"][pr_col] == 1
            p = prims[f][pr_col].astype(np.float32)
            for k in range(3):
                for side, bound in ((1, maxs[leaves, k]), (-1, mins[leaves, k])):
                    on = tri & (p[:, k] == bound)
                    idx = np.nonzero(on)[0]
                    out.append(np.stack([pr_col[idx], np.full(len(idx), vi), np.full(len(idx), k),
                                         np.full(len(idx), side), leaves[idx]], 1))
    c = np.concatenate(out).astype(np.int64)
    return np.unique(c, axis=0)


def grazing_triangle_rays(prims, mins, maxs, left, right, n=4000, seed=0, span=1.0):
    """(origins[n, 3], directions[n, 3]) f32, as the module docstring describes;
    span: the distance scale of the origins from their target point."""
    rng = np.random.default_rng(seed)
    cand = leaf_candidates(prims, mins, maxs, left, right)
    ti = cand[:, 0]
    a = prims["a"][ti].astype(np.float64)
    e1 = prims["b"][ti].astype(np.float32).astype(np.float64) - a
    e2 = prims["c"][ti].astype(np.float32).astype(np.float64) - a
    w_tri = np.linalg.norm(e1, axis=1) * np.linalg.norm(e2, axis=1)
    pick = rng.choice(len(cand), n, p=w_tri / w_tri.sum())
    c = cand[pick]
    t_idx, vi, k, side = c[:, 0], c[:, 1], c[:, 2], c[:, 3].astype(np.float64)
    A = prims["a"][t_idx].astype(np.float32)
    B = prims["b"][t_idx].astype(np.float32)
    Cc = prims["c"][t_idx].astype(np.float32)
    v = np.where(vi[:, None] == 0, A, np.where(vi[:, None] == 1, B, Cc)).astype(np.float64)
    # n = e1 x e2 in f32 as triangle.zig:35-38 computes it (the reference's det uses it)
    f = np.float32
    E1, E2 = (B - A).astype(f), (Cc - A).astype(f)
    nf = np.stack([E1[:, 1] * E2[:, 2] - E1[:, 2] * E2[:, 1], E1[:, 2] * E2[:, 0] - E1[:, 0] * E2[:, 2],
                   E1[:, 0] * E2[:, 1] - E1[:, 1] * E2[:, 0]], 1).astype(f).astype(np.float64)
    nlen = np.linalg.norm(nf, axis=1)
    nh = nf / nlen[:, None]
    # in-plane direction of s e_k (outward across L's face on axis k)
    ek = np.zeros((n, 3))
    ek[np.arange(n), k] = side
    w = ek - (ek * nh).sum(1)[:, None] * nh
    wl = np.linalg.norm(w, axis=1)
    ok = wl > 1e-3
    w = w / np.maximum(wl, 1e-30)[:, None]
    # incidence: det = -d . n in [1e-6, 1e-3] (cos theta = det / |n|, at most 0.5)
    det = 10.0 ** rng.uniform(-6, -3, n)
    cos = np.minimum(det / nlen, 0.5)
    # a random in-plane heading q, then d = cos (-n^) + sin q
    r = rng.normal(size=(n, 3))
    q = r - (r * nh).sum(1)[:, None] * nh
    q /= np.linalg.norm(q, axis=1)[:, None]
    d = -cos[:, None] * nh + np.sqrt(1.0 - cos ** 2)[:, None] * q
    dist = span * rng.uniform(0.3, 2.0, n)
    # gap g: 0.02 .. 4 x the measured reach 2.6 u |ao| |e1||e2| / det (|ao| ~ dist)
    e12 = np.linalg.norm(E1.astype(np.float64), axis=1) * np.linalg.norm(E2.astype(np.float64), axis=1)
    reach = 2.6 * U * dist * e12 / np.maximum(cos * nlen, 1e-30)
    g = reach * 10.0 ** rng.uniform(np.log10(0.02), np.log10(4.0), n)
    P = v + g[:, None] * w
    o = (P - d * dist[:, None]).astype(np.float32)
    d = d.astype(np.float32)
    keep = ok & np.all(np.isfinite(o), 1)
    return o[keep], d[keep]


def scene_span(prims):
    """The largest extent of the scene's triangles (the origin distance scale)."""
    tri = prims[prims["kind"] == 1]
    pts = np.concatenate([tri["a"], tri["b"], tri["c"]]).reshape(-1, 3)
    return float(np.max(pts.max(0) - pts.min(0)))
