"""ORACLE — test infrastructure only.

ctypes wrapper of liboracle.so, the single-threaded CPU restatement of the
reference path (see oracle.h).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg import this module; the product (zraytrace_amd)
never does.  The boundary structs come from zraytrace_amd._ffi because the
oracle consumes exactly the C-ABI scene description (include/zrt.h).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from zraytrace_amd import _ffi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    L = C.CDLL(LIB_PATH)
    S = C.POINTER(_ffi.Scene)
    f3 = C.POINTER(C.c_float)
    L.oracle_render.argtypes = [S, C.POINTER(_ffi.Camera), C.POINTER(_ffi.Params), f3,
                                C.POINTER(_ffi.Stats)]
    L.oracle_render_rows.argtypes = [S, C.POINTER(_ffi.Camera), C.POINTER(_ffi.Params),
                                     C.c_uint32, C.c_uint32, f3, C.POINTER(_ffi.Stats)]
    L.oracle_render_scanlines.argtypes = [S, C.POINTER(_ffi.Camera), C.POINTER(_ffi.Params), f3,
                                          C.POINTER(_ffi.Stats), C.POINTER(_ffi.Scanline)]
    L.oracle_bvh_build.argtypes = [S, C.POINTER(C.POINTER(_ffi.BvhNode)), C.POINTER(C.c_uint32),
                                   C.POINTER(C.c_uint32)]
    L.oracle_camera_init.argtypes = [f3, f3, f3, C.c_float, C.c_float, C.POINTER(_ffi.Camera)]
    L.oracle_camera_init.restype = None
    L.oracle_prng_u64.argtypes = [C.c_uint32, C.c_uint64, C.POINTER(C.c_uint64), C.c_int]
    L.oracle_prng_u64.restype = None
    L.oracle_prng_f32.argtypes = [C.c_uint32, C.c_uint64, f3, C.c_int]
    L.oracle_prng_f32.restype = None
    L.oracle_sample_vector.argtypes = [C.c_uint32, C.c_uint64, C.c_int, f3]
    L.oracle_sample_vector.restype = None
    L.oracle_math1.argtypes = [C.c_int, C.c_float]
    L.oracle_math1.restype = C.c_float
    L.oracle_math2.argtypes = [C.c_int, C.c_float, C.c_float]
    L.oracle_math2.restype = C.c_float
    L.oracle_ray_at.argtypes = [f3, f3, C.c_float, f3]
    L.oracle_ray_at.restype = None
    L.oracle_unit_vector.argtypes = [f3, f3]
    L.oracle_unit_vector.restype = None
    L.oracle_triangle_hit.argtypes = [f3, f3, f3, f3, f3, C.c_float, C.c_float, f3]
    L.oracle_sphere_hit.argtypes = [f3, C.c_float, f3, f3, C.c_float, C.c_float, f3]
    L.oracle_aabb_hit.argtypes = [f3, f3, f3, f3, C.c_float, C.c_float]
    L.oracle_aabb_surface_area.argtypes = [f3, f3]
    L.oracle_aabb_surface_area.restype = C.c_float
    L.oracle_texture_albedo.argtypes = [C.POINTER(_ffi.Image), C.c_float, C.c_float, C.c_float,
                                        C.c_float, f3]
    L.oracle_texture_albedo.restype = None
    L.oracle_trace.argtypes = [S, C.c_int, f3, C.c_uint32, f3, C.POINTER(C.c_int32)]
    L.oracle_bvh_test_data.argtypes = [C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, f3, f3]
    L.oracle_bvh_test_data.restype = None
    L.oracle_free.argtypes = [C.c_void_p]
    L.oracle_free.restype = None
    _lib = L
    return L


def _fp(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a, a.ctypes.data_as(C.POINTER(C.c_float))


def render(scene_view, camera, params, rows=None):
    """oracle_render[_rows]: returns (image[H, W, 3], stats dict)."""
    L = load()
    p = params.abi() if hasattr(params, "abi") else params
    out = np.zeros((p.height, p.width, 3), dtype=np.float32)
    st = _ffi.Stats()
    ptr = out.ctypes.data_as(C.POINTER(C.c_float))
    if rows is None:
        rc = L.oracle_render(scene_view, C.byref(camera), C.byref(p), ptr, C.byref(st))
    else:
        rc = L.oracle_render_rows(scene_view, C.byref(camera), C.byref(p), rows[0], rows[1], ptr,
                                  C.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle_render failed: {rc}")
    return out, st.as_dict()


def render_scanlines(scene_view, camera, params):
    """oracle_render_scanlines: (image, stats, rows uint64[H, 6]) - the deltas the
    reference's printProgress reports after each scanline (raytrace.zig:184)."""
    L = load()
    p = params.abi() if hasattr(params, "abi") else params
    out = np.zeros((p.height, p.width, 3), dtype=np.float32)
    st = _ffi.Stats()
    rows = (_ffi.Scanline * p.height)()
    rc = L.oracle_render_scanlines(scene_view, C.byref(camera), C.byref(p),
                                   out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st), rows)
    if rc != 0:
        raise RuntimeError(f"oracle_render_scanlines failed: {rc}")
    return out, st.as_dict(), np.ctypeslib.as_array(rows).view(np.uint64).reshape(p.height, 6).copy()


def bvh_build(scene_view):
    L = load()
    nodes = C.POINTER(_ffi.BvhNode)()
    n = C.c_uint32()
    depth = C.c_uint32()
    rc = L.oracle_bvh_build(scene_view, C.byref(nodes), C.byref(n), C.byref(depth))
    if rc != 0:
        raise RuntimeError(f"oracle_bvh_build failed: {rc}")
    try:
        from zraytrace_amd import nodes_to_numpy
        return nodes_to_numpy(nodes, n.value) + (depth.value,)
    finally:
        L.oracle_free(C.cast(nodes, C.c_void_p))


def trace(scene_view, use_bvh, origins, directions):
    """oracle_trace: closest hit per ray (t, +inf on a miss; surface list index, -1)."""
    L = load()
    rays = np.ascontiguousarray(np.concatenate([np.asarray(origins, np.float32).reshape(-1, 3),
                                                np.asarray(directions, np.float32).reshape(-1, 3)], axis=1))
    n = rays.shape[0]
    t = np.empty(n, np.float32)
    prim = np.empty(n, np.int32)
    f = C.POINTER(C.c_float)
    rc = L.oracle_trace(scene_view, int(bool(use_bvh)), rays.ctypes.data_as(f), n, t.ctypes.data_as(f),
                        prim.ctypes.data_as(C.POINTER(C.c_int32)))
    if rc != 0:
        raise RuntimeError(f"oracle_trace failed: {rc}")
    return t, prim


def bvh_test_data(prng, seed, n_spheres, n_rays):
    """bvh.zig:234-247 + 277-282: (spheres float32[n, 4] {x, y, z, r}, rays float32[n_rays, 6])."""
    L = load()
    sph = np.empty((n_spheres, 4), np.float32)
    rays = np.empty((n_rays, 6), np.float32)
    f = C.POINTER(C.c_float)
    L.oracle_bvh_test_data(prng, seed, n_spheres, n_rays, sph.ctypes.data_as(f), rays.ctypes.data_as(f))
    return sph, rays


def camera_init(look_from, look_at, vup, vfov, aspect):
    L = load()
    f3 = C.c_float * 3
    out = _ffi.Camera()
    L.oracle_camera_init(f3(*look_from), f3(*look_at), f3(*vup), vfov, aspect, C.byref(out))
    return out


def prng_u64(prng, seed, n):
    out = (C.c_uint64 * n)()
    load().oracle_prng_u64(prng, seed, out, n)
    return np.array(out[:], dtype=np.uint64)


def prng_f32(prng, seed, n):
    out = np.empty(n, dtype=np.float32)
    load().oracle_prng_f32(prng, seed, out.ctypes.data_as(C.POINTER(C.c_float)), n)
    return out


def sample_vector(prng, seed, which):
    out = np.empty(3, dtype=np.float32)
    load().oracle_sample_vector(prng, seed, which, out.ctypes.data_as(C.POINTER(C.c_float)))
    return out


MATH1 = {"sin": 0, "cos": 1, "acos": 2, "atan": 3, "sqrt": 4}


def math1(name, xs):
    L = load()
    return np.array([L.oracle_math1(MATH1[name], float(x)) for x in np.asarray(xs, np.float32)],
                    dtype=np.float32)


def math2(name, ys, xs):
    L = load()
    fn = {"atan2": 0, "pow": 1}[name]
    return np.array([L.oracle_math2(fn, float(y), float(x))
                     for y, x in zip(np.asarray(ys, np.float32), np.asarray(xs, np.float32))],
                    dtype=np.float32)


def ray_at(o, d, t):
    out = np.empty(3, np.float32)
    (oa, po), (da, pd) = _fp(o), _fp(d)
    load().oracle_ray_at(po, pd, t, out.ctypes.data_as(C.POINTER(C.c_float)))
    return out


def unit_vector(v):
    out = np.empty(3, np.float32)
    va, pv = _fp(v)
    load().oracle_unit_vector(pv, out.ctypes.data_as(C.POINTER(C.c_float)))
    return out


def triangle_hit(a, b, c, o, d, t_min, t_max):
    out = np.zeros(9, np.float32)
    arrs = [_fp(x) for x in (a, b, c, o, d)]
    hit = load().oracle_triangle_hit(*[p for _, p in arrs], t_min, t_max,
                                     out.ctypes.data_as(C.POINTER(C.c_float)))
    return bool(hit), out


def sphere_hit(center, radius, o, d, t_min, t_max):
    out = np.zeros(9, np.float32)
    (ca, cp), (oa, op), (da, dp) = _fp(center), _fp(o), _fp(d)
    hit = load().oracle_sphere_hit(cp, radius, op, dp, t_min, t_max,
                                   out.ctypes.data_as(C.POINTER(C.c_float)))
    return bool(hit), out


def aabb_hit(c1, c2, o, d, t_min, t_max):
    arrs = [_fp(x) for x in (c1, c2, o, d)]
    return bool(load().oracle_aabb_hit(*[p for _, p in arrs], t_min, t_max))


def aabb_surface_area(c1, c2):
    (a1, p1), (a2, p2) = _fp(c1), _fp(c2)
    return load().oracle_aabb_surface_area(p1, p2)


def texture_albedo(pixels_hw3, u_off, v_off, u, v):
    px = np.ascontiguousarray(pixels_hw3, dtype=np.float32)
    img = _ffi.Image(px.shape[1], px.shape[0], px.ctypes.data_as(C.POINTER(C.c_float)))
    out = np.empty(3, np.float32)
    load().oracle_texture_albedo(C.byref(img), u_off, v_off, u, v,
                                 out.ctypes.data_as(C.POINTER(C.c_float)))
    return out
