"""Compressed wide nodes (accel_build.hpp quantize_wide, render.hip wide_iter_q;
DESIGN.md §3 "Compressed nodes") against the oracle.

They are opt-in (ZRT_QNODES=1: measured slower than the full nodes on the C5
mesh); the tests force them on every BVH scene and on the C5 mesh,
so every adversarial ray set of the full-node traversal runs through the 64-B
nodes and their leaf records too: zrt_trace (FAST) and the path-pool render
(MODE 8, and MODE 9 with the grazing-triangle guard) must give the oracle's
answers bit for bit.

Run on an MI355X: ``pytest -m gpu``.
"""
import numpy as np
import pytest

import zraytrace_amd as z
from oracle import oracle_py as O

import test_gpu_parity as P

pytestmark = pytest.mark.gpu

FAST = z.RenderParams(1, 1, 1, 1, traversal=z.ZRT_TRAVERSAL_FAST)


@pytest.fixture
def qnodes(monkeypatch):
    monkeypatch.setenv("ZRT_QNODES", "1")


def fast_bad(scene, o, d, keep=None):
    t_ref, p_ref = O.trace(scene, True, o, d)
    t, p = z.trace(keep or scene, FAST, o, d)
    return int(((p != p_ref) | ~P.same_bits(t, t_ref)).sum()), p_ref


@pytest.mark.parametrize("which", [2, 3, 0, 4, "spheres"])
def test_qnodes_grazing_rays(scenes, which, qnodes):
    """tests/grazing_rays.py (rays in and beside box-face planes, through vertices,
    box corners and edges): the quantized boxes are larger, the leaf records hold
    the reference's planes - FAST equals the oracle."""
    keep, view, o, d = P._grazing_case(scenes, which)
    bad, p_ref = fast_bad(view, o, d, keep)
    assert (p_ref >= 0).mean() > 0.5
    assert bad == 0


@pytest.mark.parametrize("which", [2, 3, 0, 4])
def test_qnodes_grazing_triangles(scenes, which, qnodes):
    """tests/grazing_tris.py with the grazing-triangle guard (zrt_trace carries it)."""
    import grazing_tris as G
    s = scenes(which)
    pr = P.prim_array(s.view.contents)
    mins, maxs, left, right, _ = O.bvh_build(s.view)
    o, d = G.grazing_triangle_rays(pr, mins, maxs, left, right, n=20000, seed=1, span=G.scene_span(pr))
    bad, p_ref = fast_bad(s.view, o, d, s)
    assert (p_ref >= 0).mean() > 0.5
    assert bad == 0


def test_qnodes_near_miss_spheres(qnodes):
    import adversarial_rays as A
    scene, o, d = A.near_miss_scene(0)
    bad, p_ref = fast_bad(scene, o, d)
    assert (p_ref >= 0).sum() > 10000 and bad == 0


@pytest.mark.parametrize("which,scale,translate", [(2, 1.0, 1e4), (3, 1e-3, 0.0), (3, 1e3, 0.0)])
def test_qnodes_transformed_scenes(scenes, which, scale, translate, qnodes):
    """Scenes moved 10^4 away or scaled by 10^-3 / 10^3: the quantization's step and
    origin follow the coordinates' magnitude (|origin / step| < 2^24)."""
    import adversarial_rays as A
    pr = A.prim_array(scenes(which).view.contents)
    scene, o, d = A.transformed_case(O, pr, scale, translate, seed=which)
    bad, p_ref = fast_bad(scene, o, d)
    assert (p_ref >= 0).mean() > 0.2 and bad == 0


def test_qnodes_far_spheres(qnodes):
    import adversarial_rays as A
    scene, o, d = A.far_spheres_case(O, 1e4)
    bad, p_ref = fast_bad(scene, o, d)
    assert (p_ref >= 0).sum() > 300 and bad == 0


def test_qnodes_order_hazard_band(qnodes):
    import hazard_rays as H
    scene, o, d = H.hazard_scene(1, 100000)
    c = H.classify(O, scene, o, d)
    t, p = z.trace(scene, FAST, o, d)
    assert c["hazard"].sum() > 50
    P.assert_same_hits(t, p, c["t_ref"], c["p_ref"])


@pytest.mark.parametrize("which", [3, "spheres"])
def test_qnodes_per_axis_every_wave(scenes, which, qnodes, monkeypatch):
    """Every wave on the per-axis widening (ZRT_PAXIS_M=0): the leaf records take
    the same widening as the quantized slabs."""
    monkeypatch.setenv("ZRT_PAXIS_M", "0")
    keep, view, o, d = P._grazing_case(scenes, which)
    bad, _ = fast_bad(view, o, d, keep)
    assert bad == 0


@pytest.mark.parametrize("case", [c for c in P.CASES if c[0] != 1], ids=[f"scene{c[0]}" for c in P.CASES if c[0] != 1])
def test_qnodes_pool_render(scenes, case, qnodes, monkeypatch):
    """The path-pool loop over compressed nodes (MODE 8) on every BVH scene, chunks
    splitting the samples: images, counters and per-scanline counters equal the
    oracle's; zrt_stats reports 64-B nodes and the pool loop."""
    monkeypatch.setenv("ZRT_POOL", "1")
    idx, w, h, _, depth = case
    s = scenes(idx)
    p = z.RenderParams(w, h, 24, depth, sample_chunk=7)
    gpu, gs, rows = z.render_progress(s, s.camera, p)
    ref, rs, rrows = O.render_scanlines(s.view, s.camera, p)
    P.assert_bit_exact(gpu, ref)
    for k in P.COUNTERS:
        assert gs[k] == rs[k], k
    np.testing.assert_array_equal(rows, rrows)
    _, st = z.render(s, s.camera, z.RenderParams(w, h, 4, depth, flags=z.ZRT_FLAG_STATS))
    assert st["node_bytes"] == 64 and st["sampling_loop"] == 5


@pytest.mark.parametrize("scene_index", [3, 4])
def test_qnodes_guarded_render(scenes, scene_index, qnodes):
    """ZRT_FLAG_GUARD over compressed nodes (MODE 9): the oracle's frame."""
    s = scenes(scene_index)
    p = z.RenderParams(40, 32, 6, 20, sample_chunk=4, flags=z.ZRT_FLAG_GUARD)
    gpu, gs = z.render(s, s.camera, p)
    ref, rs = O.render(s.view, s.camera, z.RenderParams(40, 32, 6, 20, sample_chunk=4))
    P.assert_bit_exact(gpu, ref)
    for k in P.COUNTERS:
        assert gs[k] == rs[k], k
    assert gs["guard"] > 0.0


def test_qnodes_frame_equals_full_nodes(scenes, monkeypatch):
    """The teapot frame at 128x128 x 16 spp, depth 20 (> 4 * 10^5 rays): the pool
    loop over compressed nodes and over full nodes render the same frame."""
    monkeypatch.setenv("ZRT_POOL", "1")
    s = scenes(3)
    p = z.RenderParams(128, 128, 16, 20)
    monkeypatch.setenv("ZRT_QNODES", "0")
    full, fs = z.render(s, s.camera, p)
    monkeypatch.setenv("ZRT_QNODES", "1")
    comp, cs = z.render(s, s.camera, p)
    assert cs["rays_processed"] > 400_000
    P.assert_bit_exact(comp, full)
    for k in P.COUNTERS:
        assert cs[k] == fs[k], k


@pytest.mark.parametrize("rows", [None, "2"])
def test_qnodes_c5_substitute_depth20_vs_golden(scenes, rows, qnodes, monkeypatch):
    """Scene 6 (the 1.6 M-triangle C5 mesh, its tree past the 16-bit stack) on the
    compressed nodes: 32x32 x 2 spp at depth 20 against the oracle's golden frame,
    counters and per-scanline counters (tests/golden/c5_depth20.npz); rows="2"
    forces the stack onto its global rows past 2 LDS rows.  STATS reports 64-B nodes."""
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c5_depth20.npz"))
    w, h, spp, depth, chunk = (int(x) for x in g["params"])
    monkeypatch.setenv("ZRT_ATT_LDS_ROWS", "0")
    if rows:
        monkeypatch.setenv("ZRT_STACK_LDS_ROWS", rows)
    s = scenes(6)
    p = z.RenderParams(w, h, spp, depth, sample_chunk=chunk)
    gpu, gs, grows = z.render_progress(s, s.camera, p)
    P.assert_bit_exact(gpu, g["image"])
    for name, v in zip(g["counter_names"], g["counters"]):
        assert gs[str(name)] == int(v), name
    np.testing.assert_array_equal(grows, g["rows"])
    _, st = z.render(s, s.camera, z.RenderParams(16, 16, 1, depth, flags=z.ZRT_FLAG_STATS))
    assert st["node_bytes"] == 64


def test_qnodes_c5_grazing_triangles(scenes, qnodes):
    """The grazing-triangle set on scene 6 through the compressed nodes: equal to
    the REFERENCE traversal (which reads the reference BVH, not the wide tree)."""
    import grazing_tris as G
    s = scenes(6)
    pr = P.prim_array(s.view.contents)
    mins, maxs, left, right, _ = z.bvh_build_device(s)
    o, d = G.grazing_triangle_rays(pr, mins, maxs, left, right, n=4000, seed=2, span=G.scene_span(pr))
    t_ref, p_ref = z.trace(s, z.RenderParams(1, 1, 1, 1, traversal=z.ZRT_TRAVERSAL_REFERENCE), o, d)
    t, p = z.trace(s, FAST, o, d)
    assert (p_ref >= 0).mean() > 0.5
    P.assert_same_hits(t, p, t_ref, p_ref)
