"""Host-side tests of the product library (no kernel launches; CPU only).

* libzrt.so loads and exports every symbol include/zrt.h declares;
* scene ingestion (scenes.zig / obj_reader.zig restatement) matches the
  reference's model statistics;
* the product BVH (zrt_bvh_build) is the oracle's tree, node for node;
* the C ABI reports the reference's error cases.
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

import zraytrace_amd as z
from zraytrace_amd import _ffi
from oracle import oracle_py as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(REPO, "include", "zrt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(zrt_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = _ffi.load()
    syms = header_symbols()
    assert len(syms) >= 18
    for name in syms:
        assert hasattr(lib, name), name
    # the ctypes table covers the header exactly
    assert sorted(n for n, _, _ in _ffi.SIGNATURES) == syms


def test_abi_version_and_struct_sizes():
    lib = _ffi.load()
    assert lib.zrt_abi_version() == 2 == _ffi.ABI_VERSION
    assert b"gfx950" in lib.zrt_build_info()
    assert C.sizeof(_ffi.Prim) == 60 and C.sizeof(_ffi.Camera) == 48
    assert C.sizeof(_ffi.Params) == 64 and C.sizeof(_ffi.BvhNode) == 32


@pytest.mark.parametrize("index,n_prims", [(0, 1 + 3933), (1, 7), (2, 1 + 4968), (3, 1 + 6320), (4, 3 + 6320)])
def test_scene_sizes(scenes, index, n_prims):
    """scenes.zig + obj_reader.zig: Man 1962 quads + 6 tris + 1 pentagon -> 3933
    triangles; bunny 4968; teapot 6320 (SURVEY §2 models row)."""
    assert scenes(index).n_prims == n_prims


def test_scene_errors():
    with pytest.raises(z.ZrtError) as e:
        z.load_scene(9)
    assert e.value.code == _ffi.ZRT_E_INVALID and "UnkownSceneIndex" in str(e.value)
    with pytest.raises(z.ZrtError) as e:
        z.load_scene(5)  # goat: models/high_poly_goat.obj is not shipped
    assert e.value.code == _ffi.ZRT_E_IO


def test_obj_reader_fan_order(tmp_path):
    """obj_reader.zig:66-111: 3..6-gons fan as 0,1,2 | 2,3,0 | 3,4,0 | 4,5,0;
    'v//vn' and 'v/vt/vn' forms; CRLF lines; >6 vertices is an error."""
    p = tmp_path / "m.obj"
    p.write_bytes(b"# c\r\nv 0 0 0\r\nv 1 0 0\r\nv 1 1 0\r\nv 0 1 0\r\nv 0 2 0\nv 3 3 3\n"
                  b"vn 0 0 1\nf 1//1 2//1 3//1 4//1\nf 1/1/1 2/2/2 3/3/3 4/4/4 5/5/5 6/6/6\nf 1 2 3\n")
    prims = C.POINTER(_ffi.Prim)()
    n = C.c_uint32()
    _ffi.check(_ffi.load().zrt_obj_read(str(p).encode(), 7, C.byref(prims), C.byref(n)))
    tris = [(tuple((prims[i].a.x, prims[i].a.y)), tuple((prims[i].b.x, prims[i].b.y)),
             tuple((prims[i].c.x, prims[i].c.y))) for i in range(n.value)]
    _ffi.load().zrt_free(C.cast(prims, C.c_void_p))
    assert n.value == 2 + 4 + 1
    assert tris[0] == ((0, 0), (1, 0), (1, 1)) and tris[1] == ((1, 1), (0, 1), (0, 0))
    assert tris[3] == ((1, 1), (0, 1), (0, 0)) and tris[4] == ((0, 1), (0, 2), (0, 0))
    assert tris[5] == ((0, 2), (3, 3), (0, 0))
    bad = tmp_path / "bad.obj"
    bad.write_text("v 0 0 0\nv 1 0 0\nf 1 2\n")
    rc = _ffi.load().zrt_obj_read(str(bad).encode(), 0, C.byref(prims), C.byref(n))
    assert rc == _ffi.ZRT_E_PARSE


@pytest.mark.parametrize("index", [0, 1, 2, 3, 4])
def test_bvh_matches_oracle(scenes, index):
    """bvh.zig:62-185: the product's flat BVH equals the oracle's pointer tree
    (same topology, same boxes bit for bit, same leaf order, same depth)."""
    s = scenes(index)
    a = z.bvh_build(s)
    b = O.bvh_build(s.view)
    for x, y in zip(a[:4], b[:4]):
        np.testing.assert_array_equal(x, y)
    assert a[4] == b[4]


def test_bvh_depths(scenes):
    """SURVEY §3.2 probe: bunny 6531 nodes / depth 23, teapot 7573 / 23."""
    mins, _, _, _, depth = z.bvh_build(scenes(2))
    assert (len(mins), depth) == (6531, 23)
    mins, _, _, _, depth = z.bvh_build(scenes(3))
    assert (len(mins), depth) == (7573, 23)


def test_camera_init_matches_oracle():
    got = z.camera_init((0, 0, -0.5), (0, 0, 1), (0, 1, 0), 45.0, 1.0)
    want = O.camera_init((0, 0, -0.5), (0, 0, 1), (0, 1, 0), 45.0, 1.0)
    assert bytes(got) == bytes(want)


def test_param_validation_without_device(scenes):
    """Reference error behaviour maps to ZRT_E_*; with no GPU the HIP path
    reports ZRT_E_NODEVICE instead of silently falling back."""
    s = scenes(1)
    cam = s.camera
    with pytest.raises(z.ZrtError) as e:
        z.render(s, cam, z.RenderParams(8, 16, 1, 5))  # height > width (raytrace.zig:168)
    assert e.value.code == _ffi.ZRT_E_INVALID
    with pytest.raises(z.ZrtError) as e:
        z.render(s, cam, z.RenderParams(8, 8, 1, 5, rng_mode=z.ZRT_RNG_REFERENCE_STREAM))
    assert e.value.code == _ffi.ZRT_E_UNSUPPORTED
    with pytest.raises(z.ZrtError) as e:
        z.render(s, cam, z.RenderParams(8, 8, 70000, 5))
    assert e.value.code == _ffi.ZRT_E_INVALID
    with pytest.raises(z.ZrtError) as e:  # zrt_trace: unknown traversal, checked before the device
        z.trace(s, z.RenderParams(1, 1, 1, 1, traversal=7), [[0, 0, 0]], [[0, 0, 1]])
    assert e.value.code == _ffi.ZRT_E_INVALID
    with pytest.raises(z.ZrtError) as e:  # zrt_render_multi: empty device list
        z.render_multi(s, cam, z.RenderParams(8, 8, 1, 5), [])
    assert e.value.code == _ffi.ZRT_E_INVALID
    import torch
    if not torch.cuda.is_available():
        for call in (lambda: z.render(s, cam, z.RenderParams(8, 8, 1, 5)),
                     lambda: z.render_multi(s, cam, z.RenderParams(8, 8, 1, 5), [0, 1]),
                     lambda: z.trace(s, z.RenderParams(1, 1, 1, 1), [[0, 0, 0]], [[0, 0, 1]])):
            with pytest.raises(z.ZrtError) as e:
                call()
            assert e.value.code == _ffi.ZRT_E_NODEVICE


def test_tree_layout_mismatch_is_refused(scenes, monkeypatch):
    """a wide tree whose encoding is not the one the kernels
    decode (accel_build.hpp kLayout*, render.hip kKernelLayout) is refused with
    ZRT_E_UNSUPPORTED before anything is launched - here on CPU, where the check
    runs before the device check.  (The kernels repeat the check on the device:
    kErrLayout.)"""
    s = scenes(2)
    monkeypatch.setenv("ZRT_DEBUG_TREE_LAYOUT", "1")  # flips the sphere-slot bit of the recorded layout
    for call in (lambda: z.render(s, s.camera, z.RenderParams(8, 8, 1, 5)),
                 lambda: z.RenderContext(s, z.RenderParams(8, 8, 1, 5))):
        with pytest.raises(z.ZrtError) as e:
            call()
        assert e.value.code == _ffi.ZRT_E_UNSUPPORTED and "layout" in str(e.value)
    monkeypatch.delenv("ZRT_DEBUG_TREE_LAYOUT")
    import torch
    if not torch.cuda.is_available():  # the matching layout passes on to the device check
        with pytest.raises(z.ZrtError) as e:
            z.render(s, s.camera, z.RenderParams(8, 8, 1, 5))
        assert e.value.code == _ffi.ZRT_E_NODEVICE


def test_oracle_counters_readme_rays_per_sample(scenes):
    """README.md:50-61: scene 1 at depth 30 spends 2.1446 rays per sample; the
    oracle (reference stream) lands within 2% on a 48x48x8 sample."""
    s = scenes(1)
    img, st = O.render(s.view, s.camera, z.RenderParams(48, 48, 8, 30, rng_mode=z.ZRT_RNG_REFERENCE_STREAM))
    rps = st["rays_processed"] / st["samples_processed"]
    assert abs(rps - 2144645362 / 1e9) / 2.1446 < 0.02
    assert st["pixels_processed"] == 48 * 48 and st["samples_processed"] == 48 * 48 * 8
    # counters are consistent: samples + reflections = rays + depth hits
    assert st["samples_processed"] + st["reflections"] == st["rays_processed"] + st["recursion_depth_hits"]


def test_oracle_counter_mode_is_row_separable(scenes):
    """In counter mode every pixel has its own streams: rendering rows [8, 16)
    alone gives the same pixels as the full frame."""
    s = scenes(1)
    p = z.RenderParams(16, 16, 2, 10)
    full, _ = O.render(s.view, s.camera, p)
    part, _ = O.render(s.view, s.camera, p, rows=(8, 16))
    np.testing.assert_array_equal(full[8:16], part[8:16])


def _synthetic_scene(n, seed):
    """n primitives on a coarse lattice (many equal midpoints, +-0 coordinates,
    spheres and triangles mixed): the cases where a sort's tie order shows."""
    rng = np.random.default_rng(seed)
    prims = (_ffi.Prim * n)()
    lattice = np.array([-1.0, -0.5, -0.0, 0.0, 0.5, 1.0], np.float32)
    for i in range(n):
        p = prims[i]
        if rng.random() < 0.3:
            p.kind = _ffi.ZRT_PRIM_SPHERE
            p.center = _ffi.Vec3(*rng.choice(lattice, 3))
            p.radius = float(rng.choice([0.25, 0.5]))
        else:
            p.kind = _ffi.ZRT_PRIM_TRIANGLE
            base = rng.choice(lattice, 3)
            p.a = _ffi.Vec3(*base)
            p.b = _ffi.Vec3(*(base + rng.choice(lattice, 3)))
            p.c = _ffi.Vec3(*(base + rng.choice(lattice, 3)))
    mats = (_ffi.Material * 1)(_ffi.Material(_ffi.ZRT_MAT_LAMBERTIAN, 0, 0.0))
    texs = (_ffi.Texture * 1)(_ffi.Texture(_ffi.ZRT_TEX_COLOR, 0, _ffi.Vec3(0.5, 0.5, 0.5), 0.0, 0.0))
    scene = _ffi.Scene(prims, n, 1, mats, texs, 1, 0, None)
    scene._keep = (prims, mats, texs)
    return scene


@pytest.mark.parametrize("n,seed", [(50, 1), (3000, 2), (20000, 3)])
def test_bvh_ties_match_oracle(n, seed):
    """The radix-sorted build (one sort per axis, stable LSD radix, -0 == +0)
    equals the oracle's comparison-sort restatement of bvh.zig node for node
    on inputs full of equal keys and signed zeros."""
    s = _synthetic_scene(n, seed)
    a = z.bvh_build(C.pointer(s))
    b = O.bvh_build(C.pointer(s))
    for x, y in zip(a[:4], b[:4]):
        np.testing.assert_array_equal(x, y)
    assert a[4] == b[4]


@pytest.mark.parametrize("index", [1, 6])
def test_binary_scene_round_trip(tmp_path, index):
    """zrt_scene_write / zrt_scene_read: every array of the flat scene, the
    images and the camera come back byte for byte (the 7-spheres scene with its
    earthmap texture; the 1.6 M-triangle C5 substitute), and the BVH built from
    it is the same tree."""
    import time
    t0 = time.time()
    s = z.load_scene(index)
    t_load = time.time() - t0
    path = str(tmp_path / f"scene{index}.zrts")
    s.write(path)
    t0 = time.time()
    r = z.LoadedScene.read(path)
    t_read = time.time() - t0
    a, b = s.view.contents, r.view.contents
    assert bytes(s.camera) == bytes(r.camera)
    for name, typ in (("prims", _ffi.Prim), ("materials", _ffi.Material), ("textures", _ffi.Texture)):
        n = getattr(a, "n_" + name)
        assert getattr(b, "n_" + name) == n
        size = C.sizeof(typ) * n
        assert C.string_at(getattr(a, name), size) == C.string_at(getattr(b, name), size), name
    assert a.n_images == b.n_images
    for i in range(a.n_images):
        ia, ib = a.images[i], b.images[i]
        assert (ia.width, ia.height) == (ib.width, ib.height)
        n = 12 * ia.width * ia.height
        assert C.string_at(ia.pixels, n) == C.string_at(ib.pixels, n)
    if index == 1:
        ta = z.bvh_build(s)
        tb = z.bvh_build(r)
        for x, y in zip(ta[:4], tb[:4]):
            np.testing.assert_array_equal(x, y)
    print(f"scene {index}: built {t_load:.3f} s, read back {t_read:.3f} s")


def test_binary_scene_rejects(tmp_path):
    bad = tmp_path / "bad.zrts"
    bad.write_bytes(b"NOPE" + bytes(64))
    with pytest.raises(z.ZrtError) as e:
        z.LoadedScene.read(str(bad))
    assert e.value.code == _ffi.ZRT_E_PARSE
    s = z.load_scene(1)
    good = tmp_path / "good.zrts"
    s.write(str(good))
    data = good.read_bytes()
    (tmp_path / "cut.zrts").write_bytes(data[:-100])
    # header counts from the file are checked against its size before
    # anything is allocated (2^32 - 1 primitives would ask for 240 GB)
    huge = bytearray(data)
    huge[4 + 4 * 4: 4 + 4 * 5] = (0xFFFFFFFF).to_bytes(4, "little")  # head[4] = n_prims
    (tmp_path / "huge.zrts").write_bytes(bytes(huge))
    for name in ("cut.zrts", "huge.zrts"):
        with pytest.raises(z.ZrtError) as e:
            z.LoadedScene.read(str(tmp_path / name))
        assert e.value.code == _ffi.ZRT_E_PARSE, name
    with pytest.raises(z.ZrtError) as e:
        z.LoadedScene.read(str(tmp_path / "missing.zrts"))
    assert e.value.code == _ffi.ZRT_E_IO


def test_stats_struct_matches_header():
    """zraytrace_amd._ffi.Stats lists zrt_stats's fields (include/zrt.h) in order, so
    a field added to the C struct cannot shift the ctypes layout unnoticed."""
    import re
    with open(os.path.join(REPO, "include", "zrt.h")) as f:
        h = f.read()
    body = h[h.index("typedef struct zrt_stats {"):h.index("} zrt_stats;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = re.findall(r"\b(?:u?int(?:32|64)_t|float|double)\s+(\w+)\s*;", body)
    assert names == [n for n, _ in _ffi.Stats._fields_]



def test_u8_texel_values_by_short_division():
    """render.hip att_value decodes an 8-bit texel k as dev::div_known(k, 255,
    RN(1/255)) - q = RN(k y), r = fma(-q, 255, k), RN(r y + q) - instead of a table of
    the reference's k / 255.0f (png_image.zig:88).  Checked here with exact rational
    arithmetic for every k: the same f32 bits."""
    from fractions import Fraction as F

    def rn32(x):
        f = np.float32(float(x))
        cands = [np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))]
        return min(cands, key=lambda c: (abs(F(float(c)) - x), int(np.float32(c).view(np.uint32)) & 1))

    b = np.float32(255.0)
    y = np.float32(1.0) / b
    for k in range(256):
        a = np.float32(k)
        q = rn32(F(float(a)) * F(float(y)))
        r = rn32(F(float(a)) - F(float(q)) * F(float(b)))
        got = rn32(F(float(r)) * F(float(y)) + F(float(q)))
        assert np.float32(got).view(np.uint32) == (np.float32(k) / b).view(np.uint32), k


@pytest.mark.parametrize("index", [0, 1, 2, 3, 4])
def test_lds_plans_disjoint(scenes, index):
    """every LDS layout the launch code plans for the scene -
    list, binary, reference, lockstep / wavefront / path-pool FAST loops, 16- and
    32-bit stacks, both PRNGs, max depths 0..50 - keeps its regions (stack rows,
    top wide nodes, pool queues, the lockstep loop's parked lane state, attenuation
    rows, materials) disjoint, inside the plan and float4-aligned, and the lockstep
    plan inside its 6-block share (render.hip check_plan).  No device needed."""
    n = z.debug_lds_plans(scenes(index))
    # modes 0-2 one loop each, mode 3 lockstep / wavefront / pool (full nodes, and compressed
    # ones where the scene has a tree: their real top levels); x stk16 x prng x depth
    comp = 0 if index == 1 else 1
    assert n == (1 + 1 + 1 + 1 + 1 + 1 + comp) * 2 * 2 * 6


@pytest.mark.parametrize("index", [0, 2, 3, 4])
def test_shared_buffer_sizing_covers_every_launch(scenes, index):
    """the global rows a FAST frame's launches share - the
    attenuation rows past the LDS ones and the stack rows past the LDS ones - are
    sized (zrt_render, schedule_tiles) to cover the render launch AND its scheduling
    probe, for every loop x stack width x PRNG x node format x depth x grid
    (render.hip buffer_need / check_buffers, the same check that guards each launch).
    The sizing before commit 4072f5f (the probe reused the render's attenuation rows
    without growing them) must fail where the render keeps more LDS rows than the
    probe's 4: the wavefront loop's 12 - the round-5 GPU fault of ZRT_WF=1 on C3."""
    s = scenes(index)
    n = z.debug_buffer_plans(s)
    assert n >= 3 * 2 * 2 * 9 * 3  # lockstep, wavefront, pool (+ compressed) x stk16 x prng x depth x grid
    with pytest.raises(z.ZrtError, match="scheduling probe: needs .* attenuation-row entries.*loop 1"):
        z.debug_buffer_plans(s, legacy=True)


@pytest.mark.parametrize("index", [0, 2, 3, 4])
def test_compressed_nodes_encode_the_full_tree(scenes, index):
    """accel_build.hpp quantize_wide (DESIGN.md §3 "Compressed nodes"), on CPU: in
    every octant copy every plane decodes exactly, every slot's quantized box
    contains the full node's box, inner refs are the full node's, and every leaf
    record holds the reference leaf's box and primitive refs bit for bit - what
    wide_iter_q relies on to take wide_iter's decisions."""
    s = scenes(index)
    n = z.debug_qnodes(s)
    assert n >= 8 * 4 * 100  # 8 octant copies x 4 slots x the tree's nodes
