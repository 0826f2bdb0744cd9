"""GPU box: how many grazing-triangle rays (tests/grazing_tris.py) each traversal
gets wrong against oracle_trace, per scene, with the geometry of every miss:
det, sin(phi) |cos(theta)| of the reference's hit, how far outside its leaf box
the exact plane crossing lies against FAST's margin.  VERDICT r03 #1 asks for
the pre-fix count; the same probe after the fix must print zeros.

usage: python tools/grazing_tris_probe.py [out.json] [n_rays]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import zraytrace_amd as z  # noqa: E402
from oracle import oracle_py as O  # noqa: E402
import grazing_tris as G  # noqa: E402
from test_gpu_parity import prim_array, same_bits  # noqa: E402


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    res = {}
    for si in (2, 3, 0, 4):
        s = z.load_scene(si)
        pr = prim_array(s.view.contents)
        mins, maxs, left, right, _ = O.bvh_build(s.view)
        o, d = G.grazing_triangle_rays(pr, mins, maxs, left, right, n=n, seed=1, span=G.scene_span(pr))
        t_ref, p_ref = O.trace(s.view, True, o, d)
        row = {"rays": int(len(o)), "hits": int((p_ref >= 0).sum())}
        for name, trav in (("fast", z.ZRT_TRAVERSAL_FAST), ("binary", z.ZRT_TRAVERSAL_BINARY),
                           ("reference", z.ZRT_TRAVERSAL_REFERENCE)):
            t, p = z.trace(s, z.RenderParams(1, 1, 1, 1, traversal=trav), o, d)
            bad = np.nonzero((p != p_ref) | ~same_bits(t, t_ref))[0]
            row[name] = int(len(bad))
            if name == "fast" and len(bad):
                row["fast_examples"] = [{"o": o[i].tolist(), "d": d[i].tolist(), "ref": [int(p_ref[i]), float(t_ref[i])],
                                         "fast": [int(p[i]), float(t[i])]} for i in bad[:8]]
        res[f"scene{si}"] = row
        print(si, row.get("rays"), {k: row[k] for k in ("fast", "binary", "reference")}, flush=True)
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
