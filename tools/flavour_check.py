"""A/B diagnostic: does a build's timed kernel flavour render the same frame as its
STATS flavour (the diagnostic counters' kernel) and as the shipped library?

usage: ZRT_LIB=abvar/<v>/libzrt.so python tools/flavour_check.py [scene] [w h spp depth]
prints, for the library under test: kernel ms and the frame's sha1 of the timed and the
STATS launch, the counters of both, and (when run with ZRT_REF_LIB=<path>) whether the
frame equals that library's.
"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import zraytrace_amd as z  # noqa: E402


def main():
    a = [int(x) for x in sys.argv[1:]]
    scene_i = a[0] if a else 2
    w, h, spp, depth = a[1:5] if len(a) >= 5 else (512, 512, 64, 20)
    s = z.load_scene(scene_i)
    out = {"lib": os.environ.get("ZRT_LIB", "in-tree"), "build_id": z.build_id(), "config": [scene_i, w, h, spp, depth]}
    for name, flags in (("timed", 0), ("stats", z.ZRT_FLAG_STATS)):
        img, st = z.render(s, s.camera, z.RenderParams(w, h, spp, depth, flags=flags))
        out[name] = {"sha1": hashlib.sha1(img.tobytes()).hexdigest(), "ms": round(st["render_ms"], 2),
                     **{k: int(st[k]) for k in ("rays_processed", "reflections", "background_hits",
                                                 "recursion_depth_hits", "samples_processed")}}
    out["frames_equal"] = out["timed"]["sha1"] == out["stats"]["sha1"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
