"""Peaks from tools/gpu_ubench.sh: rocprofv3 --pmc passes over build/ubench.

usage: python tools/ubench_summary.py <gpurun_out/TAG>   (prints profiles/ubench.json's content)

Every ubench kernel is launched 6 times (the first is a warm-up); load_kernel
runs the cases l1_coalesced, l1_divergent, l2_divergent in that order.  For
each case and counter: the best counter-per-second over its timed dispatches,
and per CU / per SIMD per clock (the clock from GRBM_GUI_ACTIVE, one instance
per XCD).  peaks_per_clock, for bench.py's roofline:
  valu_insts_per_simd       best 2-source VALU class (v_add/mul_f32, v_add_u32, v_xor):
                            wave64 instructions per SIMD per clock
  valu_insts_per_simd_3src  the same for v_fma_f32 / v_max3_f32 (they issue at half that rate)
  tcp_accesses_per_cu       TCP_TOTAL_CACHE_ACCESSES_sum per CU per clock (best load case)
  l2_read_req_per_cu        TCP_TCC_READ_REQ_sum per CU per clock (l2_divergent)
  td_busy_frac_max          TD_TD_BUSY_sum per CU per clock (how close to 1 a saturating load gets)
"""
import csv
import glob
import json
import os
import sys

LOAD_CASES = ["l1_coalesced", "l1_divergent", "l2_divergent"]
N_CU, N_XCD = 256, 8


def case_of(name, k):
    base = name.split("(")[0].replace("void ", "")
    if base == "load_kernel":
        return LOAD_CASES[k // 6], k % 6
    return base, k


def main():
    d = sys.argv[1]
    best = {}
    for csvp in sorted(glob.glob(os.path.join(d, "ub*", "run_counter_collection.csv"))):
        with open(csvp) as f:
            rs = list(csv.DictReader(f))
        order = {}
        for r in sorted(rs, key=lambda r: int(r["Dispatch_Id"])):
            order.setdefault(r["Kernel_Name"], [])
            if int(r["Dispatch_Id"]) not in order[r["Kernel_Name"]]:
                order[r["Kernel_Name"]].append(int(r["Dispatch_Id"]))
        for r in rs:
            case, idx = case_of(r["Kernel_Name"], order[r["Kernel_Name"]].index(int(r["Dispatch_Id"])))
            if idx == 0:
                continue  # warm-up
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            c = best.setdefault(case, {})
            c[r["Counter_Name"]] = max(c.get(r["Counter_Name"], 0.0), float(r["Counter_Value"]) / dur)
    out = {"cases": {}}
    for case, c in best.items():
        clk = c.get("GRBM_GUI_ACTIVE", 0.0) / N_XCD
        row = {k: float(f"{v:.4e}") for k, v in sorted(c.items())}
        if clk:
            row["clock_hz"] = float(f"{clk:.4e}")
        out["cases"][case] = row
    cs = out["cases"]

    def per_clk(case, ctr, units):
        c = cs.get(case, {})
        return c.get(ctr, 0.0) / units / c["clock_hz"] if c.get("clock_hz") else 0.0
    # per-clock peaks (the clock moves with the load: 2.2-2.4 GHz), which bench.py
    # scales by the clock measured on the kernel itself
    two_src = ("valu_add_f32", "valu_mul_f32", "valu_add_u32", "valu_xor_b32")
    out["peaks_per_clock"] = {
        "valu_insts_per_simd": round(max(per_clk(k, "SQ_INSTS_VALU", N_CU * 4) for k in two_src), 4),
        "valu_insts_per_simd_3src": round(max(per_clk(k, "SQ_INSTS_VALU", N_CU * 4)
                                              for k in ("valu_fma_f32", "valu_max3_f32")), 4),
        "tcp_accesses_per_cu": round(max(per_clk(k, "TCP_TOTAL_CACHE_ACCESSES_sum", N_CU) for k in LOAD_CASES), 4),
        "tcp_accesses_per_cu_divergent": round(per_clk("l1_divergent", "TCP_TOTAL_CACHE_ACCESSES_sum", N_CU), 4),
        "l2_read_req_per_cu": round(per_clk("l2_divergent", "TCP_TCC_READ_REQ_sum", N_CU), 4),
        "td_busy_frac_max": round(max(per_clk(k, "TD_TD_BUSY_sum", N_CU) for k in LOAD_CASES), 4),
    }
    with open(os.path.join(d, "events.json")) as f:
        out["events"] = json.load(f)
    out["source"] = "tools/ubench.hip under rocprofv3 --pmc (tools/gpu_ubench.sh)"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
