"""Golden fixture for the C5 substitute (scene 6) at its real depth.

The oracle (oracle/, the C restatement pinned by the reference's KATs) renders
scene 6 at 32x32 pixels, 2 samples per pixel, max depth 20 (the C5 config's
depth), counter RNG seed 42, 1-sample chunks: about 160 s of one core (a 79 s
comparison-sort BVH build of 1.6 M triangles, then the reference's loose
left-first traversal, which visits most of the 1.9 M-node tree per ray) - too
slow for the GPU test's time limit, so the frame, its progress counters and
its per-scanline counters are stored here and the GPU test
(tests/test_gpu_parity.py::test_c5_substitute_depth20_vs_golden) compares the
HIP path with them bit for bit.

usage: python tests/golden/make_c5_golden.py   (writes tests/golden/c5_depth20.npz)
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import zraytrace_amd as z  # noqa: E402
from oracle import oracle_py as O  # noqa: E402

W, H, SPP, DEPTH, CHUNK = 32, 32, 2, 20, 1


def main():
    s = z.load_scene(6)
    p = z.RenderParams(W, H, SPP, DEPTH, sample_chunk=CHUNK)
    t = time.time()
    img, st, rows = O.render_scanlines(s.view, s.camera, p)
    print(f"oracle: {time.time() - t:.1f} s, {st['rays_processed']} rays, {st['reflections']} reflections")
    keys = ("recursion_depth_hits", "reflections", "background_hits", "rays_processed", "pixels_processed",
            "samples_processed", "bvh_nodes")
    np.savez(os.path.join(HERE, "c5_depth20.npz"), image=np.ascontiguousarray(img, np.float32),
             rows=np.asarray(rows), counters=np.array([int(st[k]) for k in keys], np.int64),
             counter_names=np.array(keys), params=np.array([W, H, SPP, DEPTH, CHUNK], np.int64))


if __name__ == "__main__":
    main()
