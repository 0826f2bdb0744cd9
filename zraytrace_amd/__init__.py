"""zraytrace_amd — MI355X (gfx950) path of zraytrace's per-pixel sampling loop.

Python host helpers over the C ABI (include/zrt.h, libzrt.so).  The reference
names carry over: ``render`` replaces raytrace.render (raytrace.zig:136-203),
``load_scene`` builds the scenes of scenes.zig:267-277 (through the C++ host
mirror in csrc/scene_io.cpp), ``RenderParams`` mirrors raytrace.zig:102-108.

There is no CPU fallback: every call that renders goes through the HIP kernel
in libzrt.so and raises ZrtError(ZRT_E_NODEVICE) without an MI355X.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import _ffi
from ._ffi import (ZRT_PRNG_XOROSHIRO128, ZRT_PRNG_XOSHIRO256, ZRT_RNG_COUNTER,  # noqa: F401
                   ZRT_RNG_REFERENCE_STREAM, ZRT_TRAVERSAL_FAST, ZRT_TRAVERSAL_REFERENCE,
                   ZRT_TRAVERSAL_BINARY, ZRT_FLAG_STATS, ZRT_FLAG_NO_SCHEDULE, ZRT_FLAG_SCANLINES, ZRT_FLAG_GUARD,
                   ZrtError, check)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASSETS = os.path.join(REPO, "assets")

SCENES = {0: "manAndBall", 1: "threeBalls", 2: "bunnyAndBall", 3: "teapotAndBall",
          4: "teapotAndBallCircle", 5: "goat"}


def lib():
    return _ffi.load()


# csrc/Makefile ID_SRC, in its order, then include/zrt.h
_ID_SRC = ("render.hip", "bvh_gpu.hip", "accel_build.cpp", "accel_build.hpp", "bvh_build.cpp", "bvh_build.hpp",
           "device_math.hpp", "zrt.hpp", "scene_io.cpp", "image_io.cpp", "cli.cpp")


def build_id() -> str:
    """zrt_build_id() of the loaded library: sha1 of the kernel sources (16 hex)
    - sha1 of the device compile flags (8)."""
    L = lib()
    if not hasattr(L, "zrt_build_id"):  # an A/B variant built from older sources (ZRT_LIB)
        return "unknown"
    return L.zrt_build_id().decode()


def build_id_of_sources() -> str:
    """The source half of zrt_build_id() recomputed from the files in the tree:
    differs from build_id()'s when libzrt.so is stale against its sources."""
    import hashlib
    h = hashlib.sha1()
    csrc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")
    for f in _ID_SRC:
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(fh.read())
    with open(os.path.join(REPO, "include", "zrt.h"), "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


@dataclass
class RenderParams:
    """raytrace.zig:102-108 plus the knobs of the GPU path."""
    width: int
    height: int
    samples_per_pixel: int
    max_depth: int
    bounded_volume_hierarchy: bool = True
    seed: int = 42
    rng_mode: int = ZRT_RNG_COUNTER
    prng: int = ZRT_PRNG_XOROSHIRO128
    traversal: int = ZRT_TRAVERSAL_FAST
    rank: int = 0
    world_size: int = 1
    device: int = 0
    sample_chunk: int = 0
    flags: int = 0

    def abi(self) -> _ffi.Params:
        p = _ffi.Params()
        p.width, p.height = self.width, self.height
        p.samples_per_pixel, p.max_depth = self.samples_per_pixel, self.max_depth
        p.bounded_volume_hierarchy = 1 if self.bounded_volume_hierarchy else 0
        p.rng_mode, p.prng, p.traversal = self.rng_mode, self.prng, self.traversal
        p.seed = self.seed
        p.rank, p.world_size, p.device = self.rank, self.world_size, self.device
        p.sample_chunk = self.sample_chunk
        p.flags = self.flags
        return p


class LoadedScene:
    """A scene of scenes.zig built by the C++ host mirror (zrt_scene_load), or
    read back from a binary scene file (zrt_scene_read, LoadedScene.read)."""

    def __init__(self, index: int, assets_dir: str = ASSETS, _path: str = None):
        L = lib()
        h = C.c_void_p()
        cam = _ffi.Camera()
        if _path is None:
            check(L.zrt_scene_load(index, assets_dir.encode(), C.byref(h), C.byref(cam)))
        else:
            check(L.zrt_scene_read(_path.encode(), C.byref(h), C.byref(cam)))
        self._h = h
        self.index = index
        self.camera = cam
        self.view = L.zrt_scene_view(h)  # POINTER(Scene)

    @classmethod
    def read(cls, path: str) -> "LoadedScene":
        """A scene written by write() (zrt_scene_read)."""
        return cls(-1, _path=path)

    def write(self, path: str):
        """The flat scene and its camera as a binary scene file (zrt_scene_write)."""
        check(lib().zrt_scene_write(self.view, C.byref(self.camera), path.encode()))

    @property
    def n_prims(self) -> int:
        return self.view.contents.n_prims

    def close(self):
        if getattr(self, "_h", None):
            lib().zrt_scene_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def load_scene(index: int, assets_dir: str = ASSETS) -> LoadedScene:
    return LoadedScene(index, assets_dir)


def camera_init(look_from, look_at, vup, vfov, aspect) -> _ffi.Camera:
    """Camera.init (camera.zig:17-35)."""
    f3 = C.c_float * 3
    out = _ffi.Camera()
    check(lib().zrt_camera_init(f3(*look_from), f3(*look_at), f3(*vup), vfov, aspect, C.byref(out)))
    return out


def render(scene, camera: _ffi.Camera, params: RenderParams):
    """raytrace.render on the GPU: returns (image[H, W, 3] f32, row 0 = bottom; stats)."""
    view = scene.view if isinstance(scene, LoadedScene) else scene
    out = np.zeros((params.height, params.width, 3), dtype=np.float32)
    st = _ffi.Stats()
    p = params.abi()
    check(lib().zrt_render(view, C.byref(camera), C.byref(p),
                           out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st)))
    return out, st.as_dict()


def _scanlines_np(rows) -> np.ndarray:
    """zrt_scanline[height] -> uint64 array [height, 6] (columns: _ffi.SCANLINE_FIELDS)."""
    return np.ctypeslib.as_array(rows).view(np.uint64).reshape(len(rows), 6).copy()


def render_progress(scene, camera: _ffi.Camera, params: RenderParams):
    """render() plus the per-scanline Progress counters of raytrace.zig:184
    (zrt_render_progress): (image, stats, rows uint64[H, 6]: recursion-limit
    hits, reflections, background hits, pixels, samples, rays of each row)."""
    view = scene.view if isinstance(scene, LoadedScene) else scene
    out = np.zeros((params.height, params.width, 3), dtype=np.float32)
    st = _ffi.Stats()
    rows = (_ffi.Scanline * params.height)()
    p = params.abi()
    check(lib().zrt_render_progress(view, C.byref(camera), C.byref(p),
                                    out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st), rows))
    return out, st.as_dict(), _scanlines_np(rows)


def render_multi(scene, camera: _ffi.Camera, params: RenderParams, devices):
    """raytrace.render over several GPUs from one process (zrt_render_multi): tiles
    dealt round-robin over `devices`, one RCCL gather to devices[0].  A device
    listed twice runs two ranks (gathered by device copies).  Same image as render()."""
    view = scene.view if isinstance(scene, LoadedScene) else scene
    out = np.zeros((params.height, params.width, 3), dtype=np.float32)
    st = _ffi.Stats()
    p = params.abi()
    devs = (C.c_uint32 * len(devices))(*devices)
    check(lib().zrt_render_multi(view, C.byref(camera), C.byref(p), devs, len(devices),
                                 out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st)))
    return out, st.as_dict()


class MultiContext:
    """Persistent multi-GPU context (zrt_multi_*): scene on every device of the
    list, RCCL communicators created once; render() = zrt_render_multi's frame."""

    def __init__(self, scene, params: RenderParams, devices):
        view = scene.view if isinstance(scene, LoadedScene) else scene
        self._scene = scene
        h = C.c_void_p()
        p = params.abi()
        devs = (C.c_uint32 * len(devices))(*devices)
        check(lib().zrt_multi_create(view, C.byref(p), devs, len(devices), C.byref(h)))
        self._h = h
        self.n_ranks = len(devices)
        self._shape = None

    def render(self, camera, params: RenderParams, copy_out: bool = True):
        """One frame.  copy_out=False leaves it on devices[0] (read it with frame()):
        returns (None, stats)."""
        st = _ffi.Stats()
        p = params.abi()
        out = np.zeros((params.height, params.width, 3), dtype=np.float32) if copy_out else None
        ptr = out.ctypes.data_as(C.POINTER(C.c_float)) if copy_out else None
        check(lib().zrt_multi_render(self._h, C.byref(camera), C.byref(p), ptr, C.byref(st)))
        self._shape = (params.height, params.width, 3)
        return out, st.as_dict()

    def frame(self) -> np.ndarray:
        """The last frame, copied from devices[0] (zrt_multi_frame)."""
        out = np.zeros(self._shape, dtype=np.float32)
        check(lib().zrt_multi_frame(self._h, out.ctypes.data_as(C.POINTER(C.c_float)), out.size))
        return out

    def rank_ms(self) -> list:
        """Each rank's render-kernel time of the last frame, ms (zrt_multi_rank_ms)."""
        out = (C.c_double * self.n_ranks)()
        check(lib().zrt_multi_rank_ms(self._h, out, self.n_ranks))
        return list(out)

    def scanlines(self, height: int) -> np.ndarray:
        """Per-scanline counters of the last render made with ZRT_FLAG_SCANLINES, summed over ranks."""
        rows = (_ffi.Scanline * height)()
        check(lib().zrt_multi_scanlines(self._h, rows, height))
        return _scanlines_np(rows)

    def close(self):
        if getattr(self, "_h", None):
            lib().zrt_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def trace(scene, params: RenderParams, origins, directions):
    """Closest hit of each ray (zrt_trace): (t float32[n], +inf on a miss; prim int32[n], -1 on a miss)."""
    view = scene.view if isinstance(scene, LoadedScene) else scene
    rays = np.ascontiguousarray(np.concatenate([np.asarray(origins, np.float32).reshape(-1, 3),
                                                np.asarray(directions, np.float32).reshape(-1, 3)], axis=1))
    n = rays.shape[0]
    t = np.empty(n, np.float32)
    prim = np.empty(n, np.int32)
    p = params.abi()
    check(lib().zrt_trace(view, C.byref(p), rays.ctypes.data_as(C.POINTER(C.c_float)), n,
                          t.ctypes.data_as(C.POINTER(C.c_float)), prim.ctypes.data_as(C.POINTER(C.c_int32))))
    return t, prim


class RenderContext:
    """Device-resident scene (zrt_ctx_*): build + upload once, render many."""

    def __init__(self, scene, params: RenderParams):
        view = scene.view if isinstance(scene, LoadedScene) else scene
        self._scene = scene  # keep the host arrays alive while the ctx exists
        h = C.c_void_p()
        p = params.abi()
        check(lib().zrt_ctx_create(view, C.byref(p), C.byref(h)))
        self._h = h

    def tile_count(self, params: RenderParams) -> int:
        n = C.c_uint32()
        p = params.abi()
        check(lib().zrt_ctx_tile_count(self._h, C.byref(p), C.byref(n)))
        return n.value

    def render_tiles(self, camera, params: RenderParams, dev_tiles: int, stream: int = 0):
        p = params.abi()
        check(lib().zrt_ctx_render_tiles(self._h, C.byref(camera), C.byref(p),
                                         C.c_void_p(dev_tiles), C.c_void_p(stream or None)))

    def assemble(self, params: RenderParams, dev_gathered: int, dev_frame: int, stream: int = 0):
        p = params.abi()
        check(lib().zrt_ctx_assemble(self._h, C.byref(p), C.c_void_p(dev_gathered),
                                     C.c_void_p(dev_frame), C.c_void_p(stream or None)))

    def sync(self):
        """Wait for the last launch; raises ZrtError on a device error (zrt_ctx_sync)."""
        check(lib().zrt_ctx_sync(self._h))

    def assemble_padded(self, params: RenderParams, dev_gathered: int, stride_tiles: int, dev_frame: int,
                        stream: int = 0):
        """Assemble from a gather of equal per-rank counts: rank r at tile r * stride_tiles."""
        p = params.abi()
        check(lib().zrt_ctx_assemble_padded(self._h, C.byref(p), C.c_void_p(dev_gathered), stride_tiles,
                                            C.c_void_p(dev_frame), C.c_void_p(stream or None)))

    def scanlines(self, height: int) -> np.ndarray:
        """This rank's per-scanline counters of the last launch (ZRT_FLAG_SCANLINES)."""
        rows = (_ffi.Scanline * height)()
        check(lib().zrt_ctx_scanlines(self._h, rows, height))
        return _scanlines_np(rows)

    def stats(self) -> dict:
        st = _ffi.Stats()
        check(lib().zrt_ctx_stats(self._h, C.byref(st)))
        return st.as_dict()

    def debug_counters(self, n: int = 48):
        out = (C.c_uint64 * n)()
        check(lib().zrt_ctx_debug_counters(self._h, out, n))
        return list(out)

    def debug_wave_times(self, cap: int = 1 << 16):
        """ZRT_PROFILE builds: array[n_waves, 2] of (start, end) 100 MHz stamps of the last launch."""
        out = np.zeros(cap, np.uint64)
        n = C.c_uint32()
        check(lib().zrt_ctx_debug_wave_times(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64)), cap, C.byref(n)))
        return out[: 2 * n.value].reshape(-1, 2).copy()

    def debug_schedule(self, cap: int = 1 << 20):
        """(probe cost per local tile, tile order) of the last launch; empty if unscheduled."""
        costs = np.zeros(cap, np.uint32)
        order = np.zeros(cap, np.uint32)
        n = C.c_uint32()
        check(lib().zrt_ctx_debug_schedule(self._h, costs.ctypes.data_as(C.POINTER(C.c_uint32)),
                                           order.ctypes.data_as(C.POINTER(C.c_uint32)), cap, C.byref(n)))
        return costs[: n.value].copy(), order[: n.value].copy()

    def kernel_ms(self) -> float:
        ms = C.c_double()
        check(lib().zrt_ctx_last_kernel_ms(self._h, C.byref(ms)))
        return ms.value

    def close(self):
        if getattr(self, "_h", None):
            lib().zrt_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def bvh_build(scene):
    """The product's BVH (zrt_bvh_build) as numpy arrays (mins, maxs, left, right, max_depth)."""
    view = scene.view if isinstance(scene, LoadedScene) else scene
    nodes = C.POINTER(_ffi.BvhNode)()
    n = C.c_uint32()
    depth = C.c_uint32()
    check(lib().zrt_bvh_build(view, C.byref(nodes), C.byref(n), C.byref(depth)))
    try:
        return nodes_to_numpy(nodes, n.value) + (depth.value,)
    finally:
        lib().zrt_free(C.cast(nodes, C.c_void_p))


def bvh_build_device(scene, device: int = 0):
    """The same BVH built on the GPU (zrt_bvh_build_device), as bvh_build returns it."""
    view = scene.view if isinstance(scene, LoadedScene) else scene
    nodes = C.POINTER(_ffi.BvhNode)()
    n = C.c_uint32()
    depth = C.c_uint32()
    check(lib().zrt_bvh_build_device(view, device, C.byref(nodes), C.byref(n), C.byref(depth)))
    try:
        return nodes_to_numpy(nodes, n.value) + (depth.value,)
    finally:
        lib().zrt_free(C.cast(nodes, C.c_void_p))


def nodes_to_numpy(nodes, n):
    dt = np.dtype([("min", "<f4", 3), ("left", "<i4"), ("max", "<f4", 3), ("right", "<i4")])
    buf = np.ctypeslib.as_array(C.cast(nodes, C.POINTER(C.c_uint8)), shape=(n * 32,)).copy()
    a = buf.view(dt)
    return a["min"].copy(), a["max"].copy(), a["left"].copy(), a["right"].copy()


def debug_division(n: int = 1 << 30, device: int = 0) -> dict:
    """Device self-check of the kernel's short correctly rounded divisions
    (zrt_debug_division): mismatch counts against HIP's IEEE `/`."""
    out = (C.c_uint64 * 5)()
    check(lib().zrt_debug_division(n, out, device))
    return dict(zip(("rcp_sqrt_all_2p32", "div", "unit", "inv_dir", "jitter"), (int(v) for v in out)))


def debug_math(fn: int, x, y=None, device: int = 0):
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(x)
    yp = None
    if y is not None:
        y = np.ascontiguousarray(y, dtype=np.float32)
        yp = y.ctypes.data_as(C.POINTER(C.c_float))
    check(lib().zrt_debug_math(fn, x.ctypes.data_as(C.POINTER(C.c_float)), yp,
                               out.ctypes.data_as(C.POINTER(C.c_float)), x.size, device))
    return out


def debug_rng(prng: int, key: int, n: int, device: int = 0):
    out = np.empty(n, dtype=np.uint64)
    check(lib().zrt_debug_rng(prng, key, out.ctypes.data_as(C.POINTER(C.c_uint64)), n, device))
    return out


def read_png(path: str):
    """png_image.readFile (zrt_image_read_png): float32[height, width, 3], row 0 = bottom, c/255."""
    w, h, px = C.c_uint32(), C.c_uint32(), C.POINTER(C.c_float)()
    check(lib().zrt_image_read_png(path.encode(), C.byref(w), C.byref(h), C.byref(px)))
    try:
        return np.ctypeslib.as_array(px, shape=(h.value, w.value, 3)).copy()
    finally:
        lib().zrt_free(px)


def write_png(path: str, image) -> None:
    """png_image.writeFile (png_image.zig:96-148) for a framebuffer[H, W, 3] (row 0 = bottom)."""
    img = np.ascontiguousarray(image, dtype=np.float32)
    h, w, _ = img.shape
    check(lib().zrt_image_write_png(os.fsencode(path), img.ctypes.data_as(C.POINTER(C.c_float)), w, h))


def write_ppm(path: str, image) -> None:
    """ppm_image.writeFile (plain P3) for a framebuffer[H, W, 3] (row 0 = bottom)."""
    img = np.ascontiguousarray(image, dtype=np.float32)
    h, w, _ = img.shape
    check(lib().zrt_image_write_ppm(os.fsencode(path), img.ctypes.data_as(C.POINTER(C.c_float)), w, h))


def debug_lds_plans(scene) -> int:
    """Host-side check of every LDS layout the launch code can plan for this scene
    (zrt_debug_lds_plans; no device): returns the number of plans checked, raises
    ZrtError naming the first overlapping / misaligned / oversized region."""
    view = scene.view if isinstance(scene, LoadedScene) else scene
    n = C.c_uint32()
    check(lib().zrt_debug_lds_plans(view, C.byref(n)))
    return n.value


def debug_buffer_plans(scene, legacy: bool = False) -> int:
    """Host-side check of the global attenuation / stack-overflow rows a FAST frame's
    launches share (zrt_debug_buffer_plans; no device): zrt_render's sizing against
    the need of the render launch and of its scheduling probe, for every loop, stack
    width, PRNG, node format and a range of depths and grids.  Returns the number of
    configurations checked, raises ZrtError naming the first launch whose rows would
    lie past its buffer.  legacy=True applies the sizing before the round-5 fix."""
    view = scene.view if isinstance(scene, LoadedScene) else scene
    n = C.c_uint32()
    check(lib().zrt_debug_buffer_plans(view, 1 if legacy else 0, C.byref(n)))
    return n.value


def debug_qnodes(scene) -> int:
    """Host-side check of the scene's compressed wide nodes (zrt_debug_qnodes; no
    device): returns the number of slots checked, raises ZrtError on a violation."""
    view = scene.view if isinstance(scene, LoadedScene) else scene
    n = C.c_uint64()
    check(lib().zrt_debug_qnodes(view, C.byref(n)))
    return n.value
