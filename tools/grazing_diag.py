"""GPU box: the grazing-ray cases of tests/test_gpu_parity.py::test_trace_grazing_rays_bit_exact
per traversal, mismatches against oracle_trace written to JSON (ray index, o, d, the
oracle's and each traversal's (t, surface)) for analysis on the CPU.

usage: python tools/grazing_diag.py <out.json> [scene ...]
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
import grazing_rays as G  # noqa: E402
from test_gpu_parity import prim_array  # noqa: E402

NAMES = {z.ZRT_TRAVERSAL_FAST: "fast", z.ZRT_TRAVERSAL_REFERENCE: "reference", z.ZRT_TRAVERSAL_BINARY: "binary"}


def main():
    out = sys.argv[1]
    which = [int(s) for s in sys.argv[2:]] or [3, 0, 4]
    res = {}
    for w in which:
        keep = z.load_scene(w)
        view = keep.view
        pr = prim_array(view.contents if hasattr(view, "contents") else view)
        mins, maxs, left, _, _ = O.bvh_build(view)
        o, d = G.grazing_rays(pr, mins, maxs, left, n=6000, seed=7, span=float(np.max(maxs[0] - mins[0])))
        t_ref, p_ref = O.trace(view, True, o, d)
        bad = set()
        per = {}
        for trav, name in NAMES.items():
            t, p = z.trace(keep, z.RenderParams(1, 1, 1, 1, traversal=trav), o, d)
            m = (p != p_ref) | (t.view(np.uint32) != t_ref.view(np.uint32))
            per[name] = (t, p)
            bad |= set(np.nonzero(m)[0].tolist())
            print(w, name, int(m.sum()), "mismatches", flush=True)
        rows = []
        for i in sorted(bad):
            row = {"i": i, "o": o[i].tolist(), "d": d[i].tolist(),
                   "oracle": [float(t_ref[i]), int(p_ref[i])]}
            for name, (t, p) in per.items():
                row[name] = [float(t[i]), int(p[i])]
            rows.append(row)
        res[str(w)] = rows
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
