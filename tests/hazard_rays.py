"""Adversarial rays for the FAST traversal's order-hazard guard (DESIGN.md §3,
"Exactness").  Test infrastructure: used by
tests/test_oracle_kat.py (CPU, pins the construction) and
tests/test_gpu_parity.py (GPU, bit-exact against oracle_trace).

Scene: a sphere of radius 100 resting on y = 0 (center (0, 100, 0), its leaf
box's bottom plane is exactly y = 0) and small downward-facing triangles just
below that plane (y = -1e-7 .. -4e-6), which the reference BVH (bvh.zig:62-185)
puts before the sphere in its DFS order.  Rays start 0.01 - 0.3 below the
sphere's lowest point and point up at it.  |oc|^2 - r^2 of such a ray
(sphere.zig:33-36) is computed from values near 10^4, whose f32 spacing is
~10^-3, so the rounded sphere hit t* scatters by ~10^-6 / h relative around the
true one and often lies BEFORE the leaf box's loose entry E (aabb.zig:109-127):
E / t* in (1 + 2^-15, 1 + 2^-14] is the band round 1's FAST did not guard.  A
triangle hit t' with t* < t' <= E in an earlier DFS leaf then makes the
reference reject the sphere's leaf and return the triangle, although the
sphere's t* is the smallest hit (bvh.zig:187-205 order effect).
"""
import ctypes as C

import numpy as np

from zraytrace_amd import _ffi

SPHERE = ((0.0, 100.0, 0.0), 100.0)


def scene_of(spheres, tris):
    """ArrayList(Surface): spheres first, then triangles, all Material.black_metal."""
    n = len(spheres) + len(tris)
    prims = (_ffi.Prim * n)()
    i = 0
    for c, r in spheres:
        prims[i].kind, prims[i].material = _ffi.ZRT_PRIM_SPHERE, 0
        prims[i].center, prims[i].radius = _ffi.Vec3(*map(float, c)), float(r)
        i += 1
    for a, b, c in tris:
        prims[i].kind, prims[i].material = _ffi.ZRT_PRIM_TRIANGLE, 0
        prims[i].a, prims[i].b, prims[i].c = (_ffi.Vec3(*map(float, v)) for v in (a, b, c))
        i += 1
    texs = (_ffi.Texture * 1)(_ffi.Texture(_ffi.ZRT_TEX_COLOR, 0, _ffi.Vec3(0, 0, 0), 0.0, 0.0))
    mats = (_ffi.Material * 1)(_ffi.Material(_ffi.ZRT_MAT_METAL, 0, 0.0))
    s = _ffi.Scene(prims, n, 1, mats, texs, 1, 0, C.cast(None, C.POINTER(_ffi.Image)))
    s._keep = (prims, mats, texs)
    return s


def hazard_scene(seed=1, n_rays=60000):
    """(scene, origins[n,3], directions[n,3]) as described above."""
    rng = np.random.default_rng(seed)
    tris = []
    for _ in range(24):
        x, z = rng.uniform(-0.06, 0.02, 2)
        y = -float(rng.choice([1e-7, 3e-7, 1e-6, 2e-6, 4e-6]))
        s = rng.uniform(0.02, 0.06)
        tris.append(((x, y, z), (x + s, y, z), (x, y, z + s)))  # e1 x e2 points down: hit from below
    scene = scene_of([SPHERE], tris)
    tx, tz = rng.uniform(-0.05, 0.05, n_rays), rng.uniform(-0.05, 0.05, n_rays)
    h = 10.0 ** rng.uniform(-2, -0.5, n_rays)
    ang, tilt = rng.uniform(0, 2 * np.pi, n_rays), rng.uniform(0.0, 2.0, n_rays)
    o = np.stack([tx + np.cos(ang) * tilt * h, -h, tz + np.sin(ang) * tilt * h], 1).astype(np.float32)
    d = (np.stack([tx, np.zeros(n_rays), tz], 1).astype(np.float32) - o).astype(np.float32)
    return scene, o, d


def unit(d):
    """Ray.init's normalisation (vector.zig:88-92) in f32."""
    d = np.asarray(d, np.float32)
    length = np.sqrt((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]).astype(np.float32)
    return (d / length[:, None]).astype(np.float32)


def loose_entry(lo, hi, o, d):
    """The loose entry of a box (aabb.zig:109-127: max over axes of max(t0, t_min)) in f32."""
    inv = (np.float32(1) / d).astype(np.float32)
    near = np.where(inv < 0, np.asarray(hi, np.float32)[None, :], np.asarray(lo, np.float32)[None, :])
    t = ((near.astype(np.float32) - o) * inv).astype(np.float32)
    return np.maximum(np.maximum(t[:, 0], t[:, 1]), np.maximum(t[:, 2], np.float32(0.001)))


def classify(O, scene, o, d):
    """Per ray, with the oracle: the reference BVH answer, the list answer (the
    smallest hit), the sphere's own t* and its leaf's loose entry E.  Returns a
    dict of arrays incl. `band` (the sphere is the smallest hit and E / t* in
    (1 + 2^-15, 1 + 2^-14]) and `hazard` (band and the reference returns a
    triangle: the sphere's leaf was rejected)."""
    t_ref, p_ref = O.trace(scene, True, o, d)
    t_list, p_list = O.trace(scene, False, o, d)
    t_s, _ = O.trace(scene_of([SPHERE], []), False, o, d)
    mins, maxs, left, right, _ = O.bvh_build(scene)
    leaf = next(i for i in range(len(left)) if left[i] < 0 and 0 in (-left[i] - 1, -right[i] - 1))
    e = loose_entry(mins[leaf], maxs[leaf], o, unit(d))
    ratio = e / t_s
    band = (p_list == 0) & (ratio > 1 + 2 ** -15) & (ratio <= 1 + 2 ** -14)
    return {"t_ref": t_ref, "p_ref": p_ref, "p_list": p_list, "ratio": ratio, "band": band,
            "hazard": band & (p_ref != 0), "order_effect": p_ref != p_list}
