"""Write profiles/latest_pmc.json (read by bench.py) from a pmc_summary.py output.

usage: python tools/make_latest_pmc.py <pmc_traffic.json> <source label> [bench config json]
Picks the timed kernel flavour (render_kernel<3, 0, false, ...>: FAST traversal,
Xoroshiro128+, no diagnostic counters) and records its corrected HBM bytes per
launch and SQ counters for the default bench config.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT = {"scene": 2, "width": 2048, "height": 2048, "spp": 1024, "max_depth": 20, "traversal": "fast",
           "sample_chunk": 32}


def main():
    src, label = sys.argv[1], sys.argv[2]
    config = json.loads(sys.argv[3]) if len(sys.argv) > 3 else DEFAULT
    with open(src) as f:
        d = json.load(f)
    main_k = [(n, k) for n, k in d["kernels"].items() if n.startswith("void zrt::render_kernel<3, 0, false")]
    assert len(main_k) == 1, list(d["kernels"])
    name, k = main_k[0]
    out = {"config": config, "kernel": name, "hbm_bytes_per_launch": k["hbm_bytes_per_launch_corrected"],
           "duration_ns": k["duration_ns"], "sq": k.get("sq"), "source": label}
    with open(os.path.join(REPO, "profiles", "latest_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
