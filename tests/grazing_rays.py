"""Grazing rays for the FAST traversal's narrowed box test (DESIGN.md §3 and §7:
"a box the ray does not cross - narrowed test with the 2^-16 margin - holds no
primitive the reference would hit").  Test infrastructure: used by
tests/test_oracle_kat.py (CPU, pins the construction) and
tests/test_gpu_parity.py (GPU, bit-exact against oracle_trace).

Every face of every box in the reference BVH (bvh.zig:62-185) and of the wide
tree built over its leaves lies in a plane through a primitive's extreme
point: a triangle's box is the min / max of its vertices (triangle.zig:33), a
sphere's is center -+ r (sphere.zig:25-26), and an inner box is the union of
its children's.  So rays are built to run IN those planes or within a few ulps
of them, through those points:

* face rays: through a triangle vertex (or a sphere's extreme point), the
  direction's component along one axis exactly 0 or +-(2^-24 .. 2^-8) of the
  others - the slab bounds of that axis are then NaN, +-inf or huge, and the
  entry / exit distances of every box touching that plane coincide with the
  hit distance;
* corner rays: through a leaf box's corners and edge midpoints (the extremes
  of different primitives on different axes), from random directions and
  from directions with a zero component;
* offset rays: the face and corner rays moved 1-4 ulps across the plane, so
  they pass just inside or just outside the box.
"""
import numpy as np


def _ulp_shift(x, k):
    """x moved k ulps (k may be negative) in f32."""
    x = np.asarray(x, np.float32)
    out = x.copy()
    for _ in range(abs(int(k))):
        out = np.nextafter(out, np.float32(np.inf) if k > 0 else np.float32(-np.inf)).astype(np.float32)
    return out


def extreme_points(prims):
    """(points[n, 3], prim index[n]): every triangle vertex, a sphere's six
    axis extremes (center +- r per axis, the points its box faces touch)."""
    pts, idx = [], []
    tri = np.nonzero(prims["kind"] == 1)[0]
    for f in ("a", "b", "c"):
        pts.append(prims[f][tri].astype(np.float32))
        idx.append(tri)
    sph = np.nonzero(prims["kind"] == 0)[0]
    for ax in range(3):
        for s in (-1.0, 1.0):
            p = prims["center"][sph].astype(np.float32).copy()
            p[:, ax] = (p[:, ax] + np.float32(s) * prims["radius"][sph]).astype(np.float32)
            pts.append(p)
            idx.append(sph)
    return np.concatenate(pts).astype(np.float32), np.concatenate(idx)


def grazing_rays(prims, mins, maxs, left, n=6000, seed=0, span=1.0):
    """(origins[m, 3], directions[m, 3]) as described in the module docstring.
    prims: the scene's zrt_prim structured array (test_gpu_parity.prim_array);
    mins / maxs / left: the reference BVH (oracle bvh_build); span: the scene's
    size, the distance origins are placed from their target point."""
    rng = np.random.default_rng(seed)
    pts, _ = extreme_points(prims)
    O, D = [], []

    def rand_dirs(m):
        d = rng.normal(size=(m, 3)).astype(np.float32)
        return d / np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)

    def add(target, d):
        dist = np.float32(span) * rng.uniform(0.2, 1.5, (len(d), 1)).astype(np.float32)
        o = (target - d * dist).astype(np.float32)
        O.append(o)
        D.append(d.astype(np.float32))

    # face rays through extreme points
    k = rng.integers(0, len(pts), n)
    ax = rng.integers(0, 3, n)
    d = rand_dirs(n)
    tiny = np.float32(2.0) ** rng.integers(-24, -7, n).astype(np.float32)
    sign = rng.choice([-1.0, 0.0, 1.0], n, p=[0.3, 0.4, 0.3]).astype(np.float32)
    d[np.arange(n), ax] = sign * tiny
    add(pts[k], d)
    # the same, moved 1-4 ulps across the face plane
    t = pts[k].copy()
    shift = rng.choice([-4, -2, -1, 1, 2, 4], n)
    for s in np.unique(shift):
        m = shift == s
        t[m, ax[m]] = _ulp_shift(t[m, ax[m]], s)
    add(t, d)
    # corner and edge-midpoint rays of leaf boxes
    leaves = np.nonzero(left < 0)[0]
    lf = leaves[rng.integers(0, len(leaves), n // 2)]
    lo, hi = mins[lf].astype(np.float32), maxs[lf].astype(np.float32)
    pick = rng.integers(0, 2, (len(lf), 3)).astype(bool)
    corner = np.where(pick, hi, lo).astype(np.float32)
    mid_ax = rng.integers(0, 3, len(lf))
    edge = corner.copy()
    edge[np.arange(len(lf)), mid_ax] = ((lo + hi) * np.float32(0.5))[np.arange(len(lf)), mid_ax]
    for target in (corner, edge):
        add(target, rand_dirs(len(lf)))
        d2 = rand_dirs(len(lf))
        d2[np.arange(len(lf)), rng.integers(0, 3, len(lf))] = 0.0
        add(target, d2)
        t = target.copy()
        a2 = rng.integers(0, 3, len(lf))
        t[np.arange(len(lf)), a2] = _ulp_shift(t[np.arange(len(lf)), a2], 1)
        add(t, d2)
    o = np.concatenate(O).astype(np.float32)
    d = np.concatenate(D).astype(np.float32)
    keep = np.all(np.isfinite(o), 1) & (np.abs(d).max(1) > 0)
    return o[keep], d[keep]
