"""Recompute bench.py's data-return model from committed files:
a bench line (its roofline.stats_shapes: the STATS launch's vector-load shape counts,
and its kernel time), a PMC entry of the same build and config (tools/pmc_summary.py
output) and profiles/ubench.json's calibrated shape costs.

usage: python tools/dr_model.py <bench_line.json> <pmc_entry.json>
prints the model (processing cycles per shape, its fraction of the launch, the PMC
check) as JSON.  No GPU needed.
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    line = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    pmc = json.load(open(sys.argv[2]))
    sh = line["roofline"].get("stats_shapes")
    if not sh:
        sys.exit("the bench line has no roofline.stats_shapes (a library without the shape counters)")
    dc = [0] * 48
    for k, i in bench.DC_SHAPES.items():
        dc[i] = sh[k]
    cfg = line["config"]
    chunk = cfg.get("sample_chunk") or 32
    n_units = ((cfg["width"] + 7) // 8) * ((cfg["height"] + 7) // 8) * ((cfg["spp"] + chunk - 1) // chunk)
    kernel_s = line["kernel_ms_avg"] / 1e3
    cache = pmc["cache"]
    dur = min(pmc["duration_ns_per_pass"]) * 1e-9
    clk = cache["GRBM_GUI_ACTIVE"] / bench.N_XCD / dur
    m = bench.data_return_model(pmc, dc, n_units, kernel_s, clk)
    m["clock_ghz"] = round(clk / 1e9, 3)
    m["bench_build_id"], m["pmc_build_id"] = line.get("build_id"), pmc.get("build_id")
    print(json.dumps(m, indent=1))


if __name__ == "__main__":
    main()
