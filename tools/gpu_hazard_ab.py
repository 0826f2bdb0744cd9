"""GPU box: FAST on tests/hazard_rays.py's adversarial rays with the library
in ZRT_LIB (e.g. the round-1 opening margin, abvar/open16) against the
oracle: how many hazard / band / order-effect rays it gets wrong."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
import zraytrace_amd as z  # noqa: E402
import hazard_rays as H  # noqa: E402
from oracle import oracle_py as O  # noqa: E402

scene, o, d = H.hazard_scene(1, 300000)
c = H.classify(O, scene, o, d)
out = {"lib": os.environ.get("ZRT_LIB", "default"), "rays": len(o)}
for name, trav in (("fast", z.ZRT_TRAVERSAL_FAST), ("binary", z.ZRT_TRAVERSAL_BINARY)):
    t, p = z.trace(scene, z.RenderParams(1, 1, 1, 1, traversal=trav), o, d)
    wrong = p != c["p_ref"]
    out[name] = {k: int((wrong & c[k]).sum()) for k in ("hazard", "band", "order_effect")}
    out[name]["all"] = int(wrong.sum())
out["counts"] = {k: int(c[k].sum()) for k in ("hazard", "band", "order_effect")}
print(json.dumps(out))
