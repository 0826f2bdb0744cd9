"""Pin the oracle (CPU restatement) to the reference's own unit-test answers.

Each test restates one reference test (file:line in the name's docstring) with
the committed fixtures of tests/golden/golden.json.  CPU only.
"""
import os

import numpy as np
import pytest

from oracle import oracle_py as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
XORO, XOSHI = 0, 1


def f32(x):
    return np.float32(x)


def test_prng_streams_match_python_emulation(golden):
    """std.rand Xoroshiro128 / Xoshiro256 seeded by SplitMix64 (bit-exact)."""
    S = golden["streams"]
    for name, prng in (("xoroshiro128", XORO), ("xoshiro256", XOSHI)):
        for seed in (0, 42, 0x123456789ABCDEF):
            want = np.array([int(v) for v in S[f"{name}_u64_seed{seed}"]], dtype=np.uint64)
            np.testing.assert_array_equal(O.prng_u64(prng, seed, 64), want)
            wantf = np.array(S[f"{name}_f32_seed{seed}"], dtype=np.float32)
            np.testing.assert_array_equal(O.prng_f32(prng, seed, 64), wantf)


def test_counter_keys(golden):
    for k in golden["streams"]["counter_keys_seed42"]:
        want = np.array([int(v) for v in k["u64"]], dtype=np.uint64)
        np.testing.assert_array_equal(O.prng_u64(XORO, int(k["key"]), 8), want)


@pytest.mark.parametrize("which,name", [(0, "randomVector"), (1, "randomVectorInUnitSphere"),
                                        (2, "randomUnitVector_old"), (3, "randomUnitVector")])
def test_sample_golden_vectors(golden, which, name):
    """sample.zig:70-118 with DefaultPrng.init(0): pins Xoroshiro128 as the generator."""
    g = golden["reference_tests"]["sample"]
    v = O.sample_vector(XORO, g["seed"], which)
    assert np.all(np.abs(v - np.array(g[name], np.float32)) < g["tol"])
    if which == 0:
        assert np.linalg.norm(v) > 1.0
    elif which == 1:
        assert np.linalg.norm(v) < 1.0
    else:
        assert 0.99 < np.linalg.norm(v) < 1.01


def test_sample_vectors_reject_xoshiro256(golden):
    """The golden vectors of sample.zig do NOT come from Xoshiro256."""
    g = golden["reference_tests"]["sample"]
    v = O.sample_vector(XOSHI, g["seed"], 0)
    assert not np.all(np.abs(v - np.array(g["randomVector"], np.float32)) < g["tol"])


def test_ray_at(golden):
    """ray.zig:32-39: Ray.init normalizes; rayAt(2) exact in f32."""
    g = golden["reference_tests"]["ray_at"]
    np.testing.assert_array_equal(O.ray_at(g["origin"], g["direction"], g["t"]),
                                  np.array(g["expected"], np.float32))


def test_unit_vector(golden):
    """vector.zig:210-225 (zero vector -> NaN)."""
    for case in golden["reference_tests"]["unit_vector"]:
        np.testing.assert_array_equal(O.unit_vector(case["v"]), np.array(case["expected"], np.float32))
    assert np.all(np.isnan(O.unit_vector([0, 0, 0])))


def test_triangle_hit_and_miss(golden):
    """triangle.zig:84-118."""
    g = golden["reference_tests"]["triangle_miss"]
    hit, _ = O.triangle_hit(g["a"], g["b"], g["c"], g["origin"], g["direction"], g["t_min"], g["t_max"])
    assert not hit
    g = golden["reference_tests"]["triangle_hit"]
    hit, out = O.triangle_hit(g["a"], g["b"], g["c"], g["origin"], g["direction"], g["t_min"], g["t_max"])
    assert hit
    np.testing.assert_array_equal(out[0:3], np.array(g["location"], np.float32))
    np.testing.assert_array_equal(out[3:6], np.array(g["normal"], np.float32))
    assert out[6] == f32(g["t"])
    assert bool(out[7]) == g["front_face"]


def test_triangle_single_sided():
    """det >= 1e-6 (triangle.zig:62): the same triangle seen from behind misses."""
    a, b, c = [10, 5, 1], [-10, -10, 1], [-10, 10, 1]
    hit, _ = O.triangle_hit(a, b, c, [0, 0, 10], [0, 0, -1], 0.1, 1e4)
    assert not hit


def test_aabb(golden):
    """aabb.zig:151-254."""
    R = golden["reference_tests"]
    g = R["aabb_surface_area"]
    assert O.aabb_surface_area(g["c1"], g["c2"]) == f32(g["expected"])
    g = R["aabb_hit"]
    for case in g["cases"]:
        assert O.aabb_hit(g["c1"], g["c2"], g["origin"], case["direction"], g["t_min"], g["t_max"]) == case["hit"]


def test_aabb_axes_tested_independently():
    """aabb.zig:120-124 tests each axis against [t_min, t_max] alone: a ray that
    passes beside a box (its x and y slab intervals do not overlap each other)
    still "hits" it.  The GPU's reference traversal mode must reproduce this."""
    # box [1,2]x[1,2]x[-1,1]; ray from origin along (1, 0.2, 0): the x-slab is
    # entered at t=1..2, the y-slab at t=5..10: disjoint, yet accepted.
    assert O.aabb_hit([1, 1, -1], [2, 2, 1], [0, 0, 0], [1, 0.2, 0], 0.001, np.inf)


def test_texture_earthmap(golden):
    """texture.zig:90-103: PNG decode (libzrt's png_image.readFile restatement)
    + row flip + c/255 + nearest texel (exact)."""
    import zraytrace_amd as z
    g = golden["reference_tests"]["texture_earthmap"]
    img = z.read_png(os.path.join(REPO, g["file"]))
    for case in g["cases"]:
        got = O.texture_albedo(img, g["u_offset"], g["v_offset"], *case["uv"])
        np.testing.assert_array_equal(got, np.array(case["expected"], np.float32))


def test_math_restatements_close_to_libm():
    """sin/cos/acos/atan/atan2/pow restatements agree with libm to a few ulp
    (they are not pinned bit-exactly to Zig: no Zig toolchain here)."""
    x = np.linspace(0, 6.2831, 997, dtype=np.float32)
    np.testing.assert_allclose(O.math1("sin", x), np.sin(x.astype(np.float64)), atol=3e-7)
    np.testing.assert_allclose(O.math1("cos", x), np.cos(x.astype(np.float64)), atol=3e-7)
    y = np.linspace(-1, 1, 1001, dtype=np.float32)
    np.testing.assert_allclose(O.math1("acos", y), np.arccos(y.astype(np.float64)), rtol=3e-7, atol=3e-7)
    np.testing.assert_allclose(O.math1("atan", y * 10), np.arctan(y.astype(np.float64) * 10), rtol=3e-7)
    ys, xs = np.meshgrid(y[::50], y[::50])
    got = O.math2("atan2", ys.ravel(), xs.ravel())
    np.testing.assert_allclose(got, np.arctan2(ys.ravel().astype(np.float64), xs.ravel()), rtol=3e-7, atol=3e-7)
    p = np.linspace(0, 2, 501, dtype=np.float32)
    np.testing.assert_allclose(O.math2("pow", p, np.full_like(p, 5.0)), p.astype(np.float64) ** 5, rtol=1e-6)
    assert O.math2("pow", [0.0], [5.0])[0] == 0.0 and O.math2("pow", [1.0], [5.0])[0] == 1.0


def test_bvh_hit_reference_test():
    """bvh.zig:262-291: 3127 random spheres, 2000 random rays from DefaultPrng(42);
    the reference asserts 10 < hits < 1500 through BVHNode.hit.  The oracle's
    reference-order traversal satisfies it and agrees with the plain surface list."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from test_gpu_parity import sphere_scene
    sph, rays = O.bvh_test_data(0, 42, 3127, 2000)
    f = O.prng_f32(0, 42, 4)  # the first sphere is the stream's first four floats
    np.testing.assert_array_equal(sph[0], np.array([(f[0] - np.float32(0.5)) * np.float32(100),
                                                    (f[1] - np.float32(0.5)) * np.float32(100),
                                                    (f[2] - np.float32(0.5)) * np.float32(100),
                                                    f[3] * np.float32(10) + np.float32(0.01)], np.float32))
    scene = sphere_scene(sph)
    t, p = O.trace(scene, True, rays[:, :3], rays[:, 3:])
    assert 10 < int((p >= 0).sum()) < 1500
    t2, p2 = O.trace(scene, False, rays[:, :3], rays[:, 3:])
    assert (p == p2).all() and ((t == t2) | (np.isinf(t) & np.isinf(t2))).all()


def test_hazard_rays_reach_the_band():
    """tests/hazard_rays.py builds the order hazard round 1's FAST left unguarded:
    the sphere's rounded hit t* is the smallest hit, its leaf's loose entry E lies
    in (t* (1 + 2^-15), t* (1 + 2^-14)], and an earlier-DFS triangle hit in
    [t*, E] makes the reference return the triangle.  Pins that the
    construction (used by the GPU parity test) produces such rays."""
    import hazard_rays as H
    scene, o, d = H.hazard_scene(1, 60000)
    c = H.classify(O, scene, o, d)
    assert c["band"].sum() > 200
    assert c["hazard"].sum() > 40
    # the reference's answer on a hazard ray is a triangle hit no closer than the sphere's
    hz = c["hazard"]
    assert (c["p_ref"][hz] > 0).all()


def test_oracle_scanlines_are_progress_deltas(scenes):
    """oracle_render_scanlines: per-row deltas of the Progress counters
    (raytrace.zig:184-186) that sum to the frame's, with raytrace.zig:168's x bound
    (height pixels per row) and the same image as oracle_render."""
    import zraytrace_amd as z
    s = scenes(1)
    p = z.RenderParams(24, 16, 4, 30)
    img, st, rows = O.render_scanlines(s.view, s.camera, p)
    ref, _ = O.render(s.view, s.camera, p)
    assert (img.view(np.uint32) == ref.view(np.uint32)).all()
    assert (rows[:, 3] == 16).all() and (rows[:, 4] == 64).all()
    assert (rows[:, 5] == rows[:, 4] + rows[:, 1] - rows[:, 0]).all()  # rays = samples + reflections - limit hits
    tot = rows.sum(axis=0)
    for i, k in enumerate(("recursion_depth_hits", "reflections", "background_hits", "pixels_processed",
                           "samples_processed", "rays_processed")):
        assert tot[i] == st[k], k


def test_grazing_rays_run_in_box_planes(scenes):
    """tests/grazing_rays.py (used by the GPU parity test of FAST's narrowed box
    test): most rays hit, over a third run exactly in an axis plane through a
    box face (a zero direction component), and the construction reaches the
    reference's order effects (BVH answer != list answer) on some of them."""
    import grazing_rays as G
    from test_gpu_parity import prim_array
    s = scenes(2)
    mins, maxs, left, _, _ = O.bvh_build(s.view)
    o, d = G.grazing_rays(prim_array(s.view.contents), mins, maxs, left, n=3000, seed=7,
                          span=float(np.max(maxs[0] - mins[0])))
    t, p = O.trace(s.view, True, o, d)
    _, pl = O.trace(s.view, False, o, d)
    assert (p >= 0).mean() > 0.5
    assert (d == 0).any(axis=1).mean() > 0.35
    assert (p != pl).sum() > 10


def test_near_miss_sphere_rays_are_accepted_outside():
    """tests/adversarial_rays.py pins its point: the reference's own sphere test
    (sphere.zig:31-41, restated by the oracle) accepts thousands of rays whose
    exact line misses the sphere - most of them outside the sphere's box too -
    so a traversal that culls boxes a ray does not cross must allow for it
    (DESIGN.md §3 "Spheres")."""
    import ctypes as C
    import adversarial_rays as A
    scene, o, d = A.near_miss_scene(0)
    _, p = O.trace(C.pointer(scene), True, o, d)
    pr = A.prim_array(scene)
    dd = A._unit(d.astype(np.float64))
    hit = np.nonzero(p >= 0)[0]
    hit = hit[pr["kind"][p[hit]] == 0]
    c = pr["center"][p[hit]].astype(np.float64)
    r = pr["radius"][p[hit]].astype(np.float64)
    oc = o[hit].astype(np.float64) - c
    hb = (oc * dd[hit]).sum(1)
    dist = np.sqrt(np.maximum((oc * oc).sum(1) - hb * hb, 0.0))
    out = dist > r
    # the exact line misses the box: outside the slab of the face the ray runs along
    q = o[hit].astype(np.float64) + dd[hit] * hb[:, None] * -1.0  # closest approach to the center
    box_miss = (np.abs(q - c) > r[:, None]).any(1)
    assert out.sum() > 3000 and (out & box_miss).sum() > 1000, (int(out.sum()), int((out & box_miss).sum()))


def test_transformed_prims_are_the_stated_map(scenes):
    """adversarial_rays.transformed_prims: v -> v * s + t per coordinate in f32."""
    import adversarial_rays as A
    pr = A.prim_array(scenes(2).view.contents)
    sph, tri = A.transformed_prims(pr, 1e3, 1e4)
    t = pr[pr["kind"] == 1][0]
    exp = (t["a"].astype(np.float32) * np.float32(1e3) + np.float32(1e4)).astype(np.float32)
    assert np.array_equal(np.asarray(tri[0][0], np.float32), exp)
    assert sph[0][1] == float(np.float32(pr[pr["kind"] == 0][0]["radius"]) * np.float32(1e3))
