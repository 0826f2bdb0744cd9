"""The rigorous reach of the rounded triangle test (triangle.zig:48-70) per
triangle of a scene, at the reference's own det floor (det >= 1e-6):

  dist(X, T) <= [8.49 u |ao| / c (2 + (|e1| + |e2|) / |e2 - e1|)
                 + 5.83 u |e1||e2| / (c |e2 - e1|) + 3 u h_a] / sin(theta_min)

X: where the exact ray crosses T's plane, c = |cos(incidence)| >= 1e-6 / |n|,
theta_min: T's smallest angle, h_a: the distance from a to bc (DESIGN.md §3
"Triangles").  Prints, per scene, the largest coefficient of |ao| and the
constant term, i.e. the spatial margin a box needs for every accepted hit of
its triangles to lie inside it grown by that much.

usage: python tools/tri_reach_bound.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def reach_coefficients(a, b, c):
    """(k_ao, k_const) per triangle: dist <= k_ao |ao| + k_const at the det floor."""
    u = 2.0 ** -24
    f = np.float32
    e1 = (b.astype(f) - a.astype(f)).astype(np.float64)
    e2 = (c.astype(f) - a.astype(f)).astype(np.float64)
    n = np.cross(e1, e2)
    nl = np.linalg.norm(n, axis=1)
    l1, l2, l3 = np.linalg.norm(e1, axis=1), np.linalg.norm(e2, axis=1), np.linalg.norm(e2 - e1, axis=1)
    # angles: at a (between e1, e2), at b, at c
    sa = nl / (l1 * l2)
    sb = nl / (l1 * l3)
    sc = nl / (l2 * l3)
    smin = np.minimum(np.minimum(sa, sb), sc)
    cmin = np.minimum(1e-6 / np.maximum(nl, 1e-300), 1.0)
    k_ao = 8.49 * u / cmin * (2.0 + (l1 + l2) / l3) / smin
    k_c = (5.83 * u * l1 * l2 / (cmin * l3) + 3 * u * nl / l3) / smin
    return k_ao, k_c, nl


def main():
    import zraytrace_amd as z
    from test_gpu_parity import prim_array
    for si in (2, 3, 0, 4, 6):
        s = z.load_scene(si)
        pr = prim_array(s.view.contents)
        tri = pr[pr["kind"] == 1]
        k_ao, k_c, nl = reach_coefficients(tri["a"], tri["b"], tri["c"])
        q = np.quantile(k_ao, [0.5, 0.9, 0.99])
        print(f"scene {si}: {len(tri)} triangles; k_ao max {k_ao.max():.3g} (2^{np.log2(k_ao.max()):.1f}), "
              f"median {q[0]:.3g}, p90 {q[1]:.3g}, p99 {q[2]:.3g}; k_const max {k_c.max():.3g}; |n| max {nl.max():.3g}")


if __name__ == "__main__":
    main()
