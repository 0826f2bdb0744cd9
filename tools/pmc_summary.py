"""Summarise tools/gpu_pmc.sh passes into the PMC entry of render_kernel.

usage: python tools/pmc_summary.py <gpurun_out/TAG>   (prints the entry as JSON)

Reads <dir>/pmcN/run_counter_collection.csv (one rocprofv3 --pmc pass each),
keeps the timed kernel flavour (render_kernel<MODE, PRNG, false, ...>: no
diagnostic counters; the one-step run launches it once), and writes per launch:
  hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1 KiB (gfx950 FETCH_SIZE
      counts half the bytes of wide reads: MI355X_MICROARCH.md §HBM),
  sq    - the SQ instruction counters and valu_lane_util
          = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU),
  cache - TCP (L1) accesses, L1->L2 read requests, TA / TD busy, GRBM_GUI_ACTIVE,
          TCC (L2) hits / misses, L2 -> memory write requests (all / 64-B ones),
and the bench config and zrt_build_id() it was measured on (from <dir>/pmc1.json,
bench's own line): bench.py attaches the entry only to that config AND that build.
"""
import csv
import glob
import json
import os
import sys


def rows(path):
    with open(path) as f:
        yield from csv.DictReader(f)


def main():
    d = sys.argv[1]
    counters, durations, names = {}, {}, set()
    for csvp in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
        for r in rows(csvp):
            name = r["Kernel_Name"]
            if "zrt::render_kernel<" not in name or ", false," not in name:
                continue  # the timed flavour only (the STATS flavour has `true`)
            names.add(name.split("(")[0])
            c = r["Counter_Name"]
            counters[c] = counters.get(c, 0.0) + float(r["Counter_Value"])
            durations.setdefault(os.path.dirname(csvp), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    assert len(names) == 1, names
    with open(os.path.join(d, "pmc1.json")) as f:
        bench = json.loads(f.read().strip().splitlines()[-1])
    cfg = {k: bench["config"][k] for k in ("scene", "width", "height", "spp", "max_depth", "traversal", "sample_chunk")}
    sq = {k: v for k, v in counters.items() if k.startswith("SQ_")}
    if sq.get("SQ_ACTIVE_INST_VALU"):
        sq["valu_lane_util"] = round(sq["SQ_THREAD_CYCLES_VALU"] / (64.0 * sq["SQ_ACTIVE_INST_VALU"]), 4)
    cache = {k: v for k, v in counters.items() if k.startswith(("TCP_", "TCC_", "TA_", "TD_", "GRBM_"))}
    entry = {"config": cfg, "build_id": bench.get("build_id"), "kernel": names.pop(),
             "hbm_bytes_per_launch": int((2 * counters["FETCH_SIZE"] + counters["WRITE_SIZE"]) * 1024),
             "fetch_size_kb": counters["FETCH_SIZE"], "write_size_kb": counters["WRITE_SIZE"],
             "duration_ns_per_pass": sorted(durations.values()),
             "sq": sq, "cache": cache, "bench_kernel_ms": bench.get("kernel_ms_avg"),
             "rays_per_launch": bench.get("rays_per_step")}
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
