"""Scenes and rays built against the FAST traversal's exactness argument
(DESIGN.md §3 "Exactness").
Test infrastructure: used by tests/test_oracle_kat.py (CPU, pins the
constructions) and tests/test_gpu_parity.py (GPU, bit-exact against
oracle_trace).

* near-miss spheres - Sphere.hit (sphere.zig:31-41) decides on the rounded
  disc = half_b^2 - (|oc|^2 - r^2), whose absolute error is ~ u |oc|^2; a ray
  that passes outside a small, distant sphere by up to ~u |oc|^2 / r (several
  per cent of r at |oc| / r ~ 10^4) is "hit", although it misses the sphere's
  box.  The rays run parallel to a box face just above the sphere's extreme
  point (where the box touches the sphere), and tangent to the sphere at small
  angles from it; some get a facing triangle just in front of the tangent point
  (near ties with the sphere's uncertain t).
* transformed scenes - the mesh scenes translated by 10^3 / 10^4 and scaled by
  10^-3 / 10^3 (every coordinate and radius in f32), traced with the grazing
  rays of tests/grazing_rays.py and random rays.
* far spheres - bvh.zig:262-291's 3127 spheres moved 10^3 / 10^4 from the
  origin.
"""
import ctypes as C

import numpy as np

import grazing_rays as G
import hazard_rays as H
from zraytrace_amd import _ffi

f32 = np.float32


def prim_array(scene):
    """A zrt_scene's prims as a numpy structured array (a view)."""
    dt = np.dtype([("kind", np.uint32), ("material", np.uint32), ("center", np.float32, 3), ("radius", np.float32),
                   ("a", np.float32, 3), ("b", np.float32, 3), ("c", np.float32, 3)])
    assert dt.itemsize == C.sizeof(_ffi.Prim)
    buf = (C.c_uint8 * (dt.itemsize * scene.n_prims)).from_address(C.addressof(scene.prims.contents))
    return np.frombuffer(buf, dtype=dt)


def _unit(v):
    v = np.asarray(v, np.float64)
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def near_miss_spheres(seed=0, n_spheres=400, n_rays=30000, extent=50.0, r_range=(0.005, 0.5),
                      dist_range=(5.0, 150.0), occluders=200):
    """(spheres [(center, r)], tris [(a, b, c)], origins[n, 3], directions[n, 3])."""
    rng = np.random.default_rng(seed)
    centers = rng.uniform(-extent, extent, (n_spheres, 3)).astype(f32)
    radii = np.exp(rng.uniform(np.log(r_range[0]), np.log(r_range[1]), n_spheres)).astype(f32)
    k = rng.integers(0, n_spheres, n_rays)
    ax = rng.integers(0, 3, n_rays)
    sgn = rng.choice([-1.0, 1.0], n_rays)
    c = centers[k].astype(np.float64)
    r = radii[k].astype(np.float64)
    e = np.zeros((n_rays, 3))
    e[np.arange(n_rays), ax] = sgn  # outward axis of the face the ray runs along
    # a random direction perpendicular to e (parallel to that box face)
    w = rng.normal(size=(n_rays, 3))
    w -= (w * e).sum(1, keepdims=True) * e
    w = _unit(w)
    kind = rng.integers(0, 3, n_rays)
    # kind 0: parallel to the face, just above / below the extreme point c + r e
    eps = rng.uniform(-0.01, 0.12, n_rays)
    p0 = c + (r * (1.0 + eps))[:, None] * e
    d0 = w + e * (rng.choice([0.0, 1.0, -1.0], n_rays) * 2.0 ** rng.uniform(-24, -8, n_rays))[:, None]
    # kind 1: tangent to the sphere at angle theta from the extreme point, in the plane of e and w
    th = rng.uniform(0.0, 0.25, n_rays)
    rad = np.cos(th)[:, None] * e + np.sin(th)[:, None] * w  # unit radius towards the tangent point
    p1 = c + (r * (1.0 + rng.uniform(-0.002, 0.02, n_rays)))[:, None] * rad
    d1 = -np.sin(th)[:, None] * e + np.cos(th)[:, None] * w  # perpendicular to the radius
    # kind 2: through a box corner region of the sphere (the box misses, the sphere is far)
    p2 = c + (r * rng.uniform(0.9, 1.05, n_rays))[:, None] * _unit(e + w)
    d2 = _unit(rng.normal(size=(n_rays, 3)))
    p = np.where(kind[:, None] == 0, p0, np.where(kind[:, None] == 1, p1, p2))
    d = _unit(np.where(kind[:, None] == 0, d0, np.where(kind[:, None] == 1, d1, d2)))
    dist = rng.uniform(*dist_range, n_rays)
    o = (p - d * dist[:, None]).astype(f32)
    spheres = [(tuple(map(float, centers[i])), float(radii[i])) for i in range(n_spheres)]
    tris = []
    # facing triangles just in front of some tangent points: near ties with the
    # sphere's rounded t (hit by the ray that placed them: det = -d.n > 0)
    for i in rng.choice(np.nonzero(kind == 1)[0], min(occluders, int((kind == 1).sum())), replace=False):
        t_hit = dist[i] * (1.0 - 10.0 ** rng.uniform(-6, -2.5))
        q = o[i].astype(np.float64) + d[i] * t_hit
        s = r[i] * 0.05
        u = _unit(np.cross(d[i], [0.3, 0.5, 0.7]))
        v = np.cross(d[i], u)
        a = q - s * u - s * v
        b = q + s * u - s * v
        cc = q + 2 * s * v
        if np.dot(np.cross(b - a, cc - a), d[i]) > 0:  # single-sided: the face normal against the ray
            b, cc = cc, b
        tris.append((tuple(map(float, a)), tuple(map(float, b)), tuple(map(float, cc))))
    return spheres, tris, o, d.astype(f32)


def near_miss_scene(seed=0, **kw):
    """(scene, origins, directions) of near_miss_spheres."""
    spheres, tris, o, d = near_miss_spheres(seed, **kw)
    return H.scene_of(spheres, tris), o, d


def transformed_prims(pr, scale=1.0, translate=0.0):
    """(spheres, tris) of a zrt_prim array with every coordinate v -> v * scale + translate
    and every radius r -> r * scale, in f32 (the order of operations the list states)."""
    s, t = f32(scale), f32(translate)
    spheres, tris = [], []
    for p in pr:
        if p["kind"] == 0:
            c = (p["center"].astype(f32) * s + t).astype(f32)
            spheres.append((tuple(map(float, c)), float(f32(p["radius"]) * s)))
        else:
            vs = [tuple(map(float, (p[n].astype(f32) * s + t).astype(f32))) for n in ("a", "b", "c")]
            tris.append(tuple(vs))
    return spheres, tris


def transformed_case(O, pr, scale, translate, seed=0, n=4000):
    """(scene, origins, directions): the scene transformed, with the grazing rays of
    tests/grazing_rays.py on it and random rays from around it."""
    spheres, tris = transformed_prims(pr, scale, translate)
    scene = H.scene_of(spheres, tris)
    mins, maxs, left, _, _ = O.bvh_build(C.pointer(scene))
    tpr = prim_array(scene)
    # the mesh part's extent sets the rays' scale (the ground sphere's box is far larger)
    tri = tpr[tpr["kind"] == 1]
    if len(tri):
        vv = np.concatenate([tri["a"], tri["b"], tri["c"]]).astype(np.float64)
    else:
        vv = tpr["center"].astype(np.float64)
    lo, hi = vv.min(0), vv.max(0)
    span = float(np.max(hi - lo))
    o1, d1 = G.grazing_rays(tpr, mins, maxs, left, n=n, seed=seed, span=span)
    rng = np.random.default_rng(seed + 1)
    o2 = rng.uniform(lo - (hi - lo), hi + (hi - lo), (n, 3)).astype(f32)
    tgt = rng.uniform(lo, hi, (n, 3))
    d2 = (tgt - o2).astype(f32)
    keep = np.abs(d2).max(1) > 0
    o = np.concatenate([o1, o2[keep]]).astype(f32)
    d = np.concatenate([d1, d2[keep]]).astype(f32)
    return scene, o, d


def far_spheres_case(O, translate, seed=0, n=4000):
    """bvh.zig:262-291's 3127 spheres (DefaultPrng(42)) moved by `translate` on every
    axis, its own 2000 random rays moved with them, plus grazing rays."""
    sph, rays = O.bvh_test_data(0, 42, 3127, 2000)  # ZRT_PRNG_XOROSHIRO128
    t = f32(translate)
    spheres = [(tuple(map(float, (np.asarray(s[:3], f32) + t).astype(f32))), float(s[3])) for s in sph]
    scene = H.scene_of(spheres, [])
    mins, maxs, left, _, _ = O.bvh_build(C.pointer(scene))
    tpr = prim_array(scene)
    o1, d1 = G.grazing_rays(tpr, mins, maxs, left, n=n, seed=seed, span=100.0)
    o2 = (rays[:, :3].astype(f32) + t).astype(f32)
    d2 = rays[:, 3:].astype(f32)
    return scene, np.concatenate([o1, o2]).astype(f32), np.concatenate([d1, d2]).astype(f32)
