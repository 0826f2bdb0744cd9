"""Recompute bench.py's data-return model from committed files:
a bench line (its roofline.stats_shapes: the STATS launch's vector-load shape counts,
and its kernel time), a PMC entry of the same build and config (tools/pmc_summary.py
output) and profiles/ubench.json's calibrated shape costs.

usage: python tools/dr_model.py [--ceilings] <bench_line.json> <pmc_entry.json>
prints the model (processing cycles per shape, its fraction of the launch, the PMC
check) as JSON; --ceilings: bench.py's whole roofline object instead (every ceiling,
the bound, the model), as a line of that build would carry it once the entry is in
profiles/latest_pmc.json.  No GPU needed.
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if a != "--ceilings"]
    line = json.loads([ln for ln in open(args[0]) if ln.startswith("{")][-1])
    pmc = json.load(open(args[1]))
    if line.get("build_id") != pmc.get("build_id"):
        sys.exit(f"build ids differ: bench line {line.get('build_id')}, PMC entry {pmc.get('build_id')}")
    sh = line["roofline"].get("stats_shapes")
    cfg = line["config"]
    chunk = cfg.get("sample_chunk") or 32
    n_units = ((cfg["width"] + 7) // 8) * ((cfg["height"] + 7) // 8) * ((cfg["spp"] + chunk - 1) // chunk)
    kernel_s = line["kernel_ms_avg"] / 1e3
    dc = None
    if sh:
        dc = [0] * 48
        for k, i in bench.DC_SHAPES.items():
            dc[i] = sh[k]
    if "--ceilings" in sys.argv:
        alg = line["roofline"]["algorithmic"]
        rays = line["rays_per_step"]
        per = alg["per_ray"]
        diag = {"rays_processed": rays, "node_visits": per["node_visits"] * rays,
                "leaf_visits": per["leaf_visits"] * rays, "prim_tests": per["prim_tests"] * rays}
        r = bench.roofline(pmc, kernel_s, alg["bytes_per_launch"], diag,
                           model_in=(dc, n_units) if dc else None)
        print(json.dumps(r, indent=1))
        return
    if not sh:
        sys.exit("the bench line has no roofline.stats_shapes (a loop without the shape counters)")
    cache = pmc["cache"]
    dur = min(pmc["duration_ns_per_pass"]) * 1e-9
    clk = cache["GRBM_GUI_ACTIVE"] / bench.N_XCD / dur
    m = bench.data_return_model(pmc, dc, n_units, kernel_s, clk)
    m["clock_ghz"] = round(clk / 1e9, 3)
    m["bench_build_id"], m["pmc_build_id"] = line.get("build_id"), pmc.get("build_id")
    print(json.dumps(m, indent=1))


if __name__ == "__main__":
    main()
