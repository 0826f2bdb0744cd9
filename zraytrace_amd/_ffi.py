"""ctypes view of include/zrt.h (the C ABI of libzrt.so).

The structures mirror the header field for field; `load()` opens the in-tree
``zraytrace_amd/libzrt.so`` built by ``__graft_entry__.build()`` and fails
loudly when it is missing: there is no Python or CPU fallback for the HIP path.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# ZRT_LIB overrides the library path (A/B of build variants, tools/variants.sh)
LIB_PATH = os.environ.get("ZRT_LIB") or os.path.join(HERE, "libzrt.so")

# ---- status / enums (zrt.h) --------------------------------------------------
ABI_VERSION = 2  # ZRT_ABI_VERSION: the layouts below (zrt_stats gained sampling_loop in 2)
ZRT_OK = 0
ZRT_E_INVALID = -1
ZRT_E_NOMEM = -2
ZRT_E_HIP = -3
ZRT_E_UNSUPPORTED = -4
ZRT_E_NODEVICE = -5
ZRT_E_IO = -6
ZRT_E_PARSE = -7

ZRT_PRIM_SPHERE, ZRT_PRIM_TRIANGLE = 0, 1
ZRT_MAT_LAMBERTIAN, ZRT_MAT_METAL, ZRT_MAT_DIELECTRIC = 0, 1, 2
ZRT_TEX_COLOR, ZRT_TEX_IMAGE = 0, 1
ZRT_RNG_COUNTER, ZRT_RNG_REFERENCE_STREAM = 0, 1
ZRT_PRNG_XOROSHIRO128, ZRT_PRNG_XOSHIRO256 = 0, 1
ZRT_TRAVERSAL_FAST, ZRT_TRAVERSAL_REFERENCE, ZRT_TRAVERSAL_BINARY = 0, 1, 2
ZRT_FLAG_STATS = 1
ZRT_FLAG_NO_SCHEDULE = 2
ZRT_FLAG_SCANLINES = 4
ZRT_FLAG_GUARD = 8


class Vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class Camera(C.Structure):
    _fields_ = [("origin", Vec3), ("lower_left_corner", Vec3),
                ("horizontal", Vec3), ("vertical", Vec3)]


class Prim(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("material", C.c_uint32), ("center", Vec3),
                ("radius", C.c_float), ("a", Vec3), ("b", Vec3), ("c", Vec3)]


class Material(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("texture", C.c_uint32),
                ("index_of_refraction", C.c_float)]


class Texture(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("image", C.c_uint32), ("color", Vec3),
                ("u_offset", C.c_float), ("v_offset", C.c_float)]


class Image(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32),
                ("pixels", C.POINTER(C.c_float))]


class Scene(C.Structure):
    _fields_ = [("prims", C.POINTER(Prim)), ("n_prims", C.c_uint32),
                ("n_materials", C.c_uint32), ("materials", C.POINTER(Material)),
                ("textures", C.POINTER(Texture)), ("n_textures", C.c_uint32),
                ("n_images", C.c_uint32), ("images", C.POINTER(Image))]


class Params(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32),
                ("samples_per_pixel", C.c_uint32), ("max_depth", C.c_uint32),
                ("bounded_volume_hierarchy", C.c_uint32), ("rng_mode", C.c_uint32),
                ("prng", C.c_uint32), ("traversal", C.c_uint32), ("seed", C.c_uint64),
                ("rank", C.c_uint32), ("world_size", C.c_uint32),
                ("device", C.c_uint32), ("sample_chunk", C.c_uint32),
                ("flags", C.c_uint32), ("reserved", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("recursion_depth_hits", C.c_uint64), ("reflections", C.c_uint64),
                ("background_hits", C.c_uint64), ("pixels_processed", C.c_uint64),
                ("samples_processed", C.c_uint64), ("rays_processed", C.c_uint64),
                ("node_visits", C.c_uint64), ("prim_tests", C.c_uint64),
                ("sphere_tests", C.c_uint64), ("shade_fetches", C.c_uint64),
                ("texel_fetches", C.c_uint64), ("leaf_visits", C.c_uint64),
                ("preprocess_ms", C.c_double), ("upload_ms", C.c_double),
                ("render_ms", C.c_double), ("gather_ms", C.c_double),
                ("used_bvh", C.c_uint32), ("bvh_nodes", C.c_uint32),
                ("bvh_max_depth", C.c_uint32), ("n_gpus", C.c_uint32),
                ("node_bytes", C.c_uint32), ("wide_nodes", C.c_uint32),
                ("texel_bytes", C.c_uint32), ("schedule_ms", C.c_float),
                ("order_replays", C.c_uint64), ("box_excess_max_triangle", C.c_float),
                ("box_excess_max_sphere", C.c_float), ("box_excess_hits", C.c_uint64),
                ("sampling_loop", C.c_uint32), ("guard", C.c_float)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


class Scanline(C.Structure):
    _fields_ = [("recursion_depth_hits", C.c_uint64), ("reflections", C.c_uint64),
                ("background_hits", C.c_uint64), ("pixels", C.c_uint64), ("samples", C.c_uint64),
                ("rays", C.c_uint64)]


SCANLINE_FIELDS = [name for name, _ in Scanline._fields_]


class BvhNode(C.Structure):
    _fields_ = [("min", Vec3), ("left", C.c_int32), ("max", Vec3), ("right", C.c_int32)]


# Every symbol include/zrt.h declares: (name, restype, argtypes)
_P = C.c_void_p
SIGNATURES = [
    ("zrt_render", C.c_int, [C.POINTER(Scene), C.POINTER(Camera), C.POINTER(Params),
                             C.POINTER(C.c_float), C.POINTER(Stats)]),
    ("zrt_render_progress", C.c_int, [C.POINTER(Scene), C.POINTER(Camera), C.POINTER(Params),
                                      C.POINTER(C.c_float), C.POINTER(Stats), C.POINTER(Scanline)]),
    ("zrt_render_multi", C.c_int, [C.POINTER(Scene), C.POINTER(Camera), C.POINTER(Params),
                                   C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_float), C.POINTER(Stats)]),
    ("zrt_multi_create", C.c_int, [C.POINTER(Scene), C.POINTER(Params), C.POINTER(C.c_uint32), C.c_uint32,
                                   C.POINTER(_P)]),
    ("zrt_multi_render", C.c_int, [_P, C.POINTER(Camera), C.POINTER(Params), C.POINTER(C.c_float),
                                   C.POINTER(Stats)]),
    ("zrt_multi_destroy", C.c_int, [_P]),
    ("zrt_multi_scanlines", C.c_int, [_P, C.POINTER(Scanline), C.c_uint32]),
    ("zrt_multi_frame", C.c_int, [_P, C.POINTER(C.c_float), C.c_uint64]),
    ("zrt_multi_rank_ms", C.c_int, [_P, C.POINTER(C.c_double), C.c_uint32]),
    ("zrt_trace", C.c_int, [C.POINTER(Scene), C.POINTER(Params), C.POINTER(C.c_float), C.c_uint32,
                            C.POINTER(C.c_float), C.POINTER(C.c_int32)]),
    ("zrt_camera_init", C.c_int, [C.POINTER(C.c_float), C.POINTER(C.c_float),
                                  C.POINTER(C.c_float), C.c_float, C.c_float,
                                  C.POINTER(Camera)]),
    ("zrt_last_error", C.c_char_p, []),
    ("zrt_abi_version", C.c_int, []),
    ("zrt_build_info", C.c_char_p, []),
    ("zrt_build_id", C.c_char_p, []),
    ("zrt_ctx_create", C.c_int, [C.POINTER(Scene), C.POINTER(Params), C.POINTER(_P)]),
    ("zrt_ctx_destroy", C.c_int, [_P]),
    ("zrt_ctx_tile_count", C.c_int, [_P, C.POINTER(Params), C.POINTER(C.c_uint32)]),
    ("zrt_ctx_render_tiles", C.c_int, [_P, C.POINTER(Camera), C.POINTER(Params), _P, _P]),
    ("zrt_ctx_assemble", C.c_int, [_P, C.POINTER(Params), _P, _P, _P]),
    ("zrt_ctx_assemble_padded", C.c_int, [_P, C.POINTER(Params), _P, C.c_uint32, _P, _P]),
    ("zrt_ctx_sync", C.c_int, [_P]),
    ("zrt_ctx_scanlines", C.c_int, [_P, C.POINTER(Scanline), C.c_uint32]),
    ("zrt_ctx_stats", C.c_int, [_P, C.POINTER(Stats)]),
    ("zrt_ctx_last_kernel_ms", C.c_int, [_P, C.POINTER(C.c_double)]),
    ("zrt_ctx_debug_counters", C.c_int, [_P, C.POINTER(C.c_uint64), C.c_uint32]),
    ("zrt_ctx_debug_wave_times", C.c_int, [_P, C.POINTER(C.c_uint64), C.c_uint32, C.POINTER(C.c_uint32)]),
    ("zrt_ctx_debug_schedule", C.c_int, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_uint32,
                                         C.POINTER(C.c_uint32)]),
    ("zrt_scene_load", C.c_int, [C.c_uint32, C.c_char_p, C.POINTER(_P), C.POINTER(Camera)]),
    ("zrt_scene_view", C.POINTER(Scene), [_P]),
    ("zrt_scene_free", None, [_P]),
    ("zrt_scene_write", C.c_int, [C.POINTER(Scene), C.POINTER(Camera), C.c_char_p]),
    ("zrt_scene_read", C.c_int, [C.c_char_p, C.POINTER(_P), C.POINTER(Camera)]),
    ("zrt_obj_read", C.c_int, [C.c_char_p, C.c_uint32, C.POINTER(C.POINTER(Prim)),
                               C.POINTER(C.c_uint32)]),
    ("zrt_free", None, [_P]),
    ("zrt_image_read_png", C.c_int, [C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                     C.POINTER(C.POINTER(C.c_float))]),
    ("zrt_image_write_png", C.c_int, [C.c_char_p, C.POINTER(C.c_float), C.c_uint32, C.c_uint32]),
    ("zrt_image_write_ppm", C.c_int, [C.c_char_p, C.POINTER(C.c_float), C.c_uint32, C.c_uint32]),
    ("zrt_bvh_build", C.c_int, [C.POINTER(Scene), C.POINTER(C.POINTER(BvhNode)),
                                C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    ("zrt_bvh_build_device", C.c_int, [C.POINTER(Scene), C.c_uint32, C.POINTER(C.POINTER(BvhNode)),
                                       C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    ("zrt_debug_math", C.c_int, [C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float),
                                 C.POINTER(C.c_float), C.c_uint32, C.c_uint32]),
    ("zrt_debug_rng", C.c_int, [C.c_uint32, C.c_uint64, C.POINTER(C.c_uint64),
                                C.c_uint32, C.c_uint32]),
    ("zrt_debug_division", C.c_int, [C.c_uint64, C.POINTER(C.c_uint64), C.c_uint32]),
    ("zrt_debug_lds_plans", C.c_int, [C.POINTER(Scene), C.POINTER(C.c_uint32)]),
    ("zrt_debug_buffer_plans", C.c_int, [C.POINTER(Scene), C.c_uint32, C.POINTER(C.c_uint32)]),
    ("zrt_debug_qnodes", C.c_int, [C.POINTER(Scene), C.POINTER(C.c_uint64)]),
]

_lib = None


class ZrtError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"zrt error {code}: {msg}")
        self.code = code


def load(path: str = LIB_PATH):
    """Open libzrt.so (the HIP path).  Raises if it was not built."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    # One HIP runtime per process: libzrt.so and torch both NEED
    # libamdhip64.so.7, and torch ships its own copy (with its own HSA runtime).
    # Whichever is loaded first is the one the process uses, and a second HSA
    # runtime cannot open the GPU.  Load torch's first so device buffers, streams
    # and RCCL (torch.distributed) share the runtime libzrt launches on.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build the HIP extension first "
            "(python -c 'import __graft_entry__ as g; g.build()'); there is no fallback path")
    lib = C.CDLL(path)
    in_tree = path == os.path.join(HERE, "libzrt.so")
    rebuild = "rebuild it (python -c 'import __graft_entry__ as g; g.build()')"
    # the ABI version first (every version exports zrt_abi_version): the struct
    # layouts below are this version's, so another version is refused before any
    # symbol is bound - an A/B variant under ZRT_LIB too (its Params / Stats would be
    # read with this version's layouts), unless ZRT_ALLOW_ABI_MISMATCH=1 asks for it
    lib.zrt_abi_version.restype = C.c_int
    lib.zrt_abi_version.argtypes = []
    abi = lib.zrt_abi_version()
    if abi != ABI_VERSION:
        if in_tree:
            raise ImportError(f"{path} has ABI version {abi}, this binding expects {ABI_VERSION}: {rebuild}")
        if os.environ.get("ZRT_ALLOW_ABI_MISMATCH") != "1":
            raise ImportError(f"ZRT_LIB {path} has ABI version {abi}, this binding expects {ABI_VERSION} "
                              "(set ZRT_ALLOW_ABI_MISMATCH=1 to bind it anyway)")
        import warnings
        warnings.warn(f"ZRT_LIB {path} has ABI version {abi}, this binding expects {ABI_VERSION} "
                      "(bound anyway: ZRT_ALLOW_ABI_MISMATCH=1)")
    for name, restype, argtypes in SIGNATURES:
        if not hasattr(lib, name):
            if in_tree:
                raise ImportError(f"{path} does not export {name} (built from older sources): {rebuild}")
            continue  # an older A/B build variant (ZRT_LIB) may lack newer entry points
        fn = getattr(lib, name)
        fn.restype = restype
        fn.argtypes = argtypes
    if path == LIB_PATH:
        _lib = lib
    return lib


def check(rc: int):
    if rc != ZRT_OK:
        raise ZrtError(rc, (load().zrt_last_error() or b"").decode())
    return rc
