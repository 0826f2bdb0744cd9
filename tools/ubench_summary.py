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


def shapes_summary(d):
    """tools/ubench_shapes.hip under rocprofv3 --pmc (passes sh1..shN): every case is
    its own kernel, launched 6 times in the order of events_shapes.json (the first a
    warm-up).  Per case: the PMC counts per timed dispatch, and per vector-memory
    wave-instruction: TD and TA busy cycles (per CU), TCP accesses, L1 -> L2 requests;
    with the HIP-event time: CU cycles per instruction at the clock the pass saw."""
    ev_path = os.path.join(d, "events_shapes.json")
    if not os.path.exists(ev_path):
        return None
    with open(ev_path) as f:
        ev = json.load(f)
    names = list(ev["shapes"].keys())
    per = {}
    for csvp in sorted(glob.glob(os.path.join(d, "sh*", "run_counter_collection.csv"))):
        with open(csvp) as f:
            rs = list(csv.DictReader(f))
        # (the runtime's own kernels - hipMemset's fill - are not cases)
        rs = [r for r in rs if not r["Kernel_Name"].lstrip().startswith("__amd")]
        first = {}
        for r in rs:
            k, i = r["Kernel_Name"].split("(")[0], int(r["Dispatch_Id"])
            first[k] = min(first.get(k, i), i)
        kernels = sorted(first, key=first.get)
        disp = {}
        for r in sorted(rs, key=lambda r: int(r["Dispatch_Id"])):
            k = r["Kernel_Name"].split("(")[0]
            disp.setdefault(k, [])
            if int(r["Dispatch_Id"]) not in disp[k]:
                disp[k].append(int(r["Dispatch_Id"]))
        for r in rs:
            k = r["Kernel_Name"].split("(")[0]
            if k not in kernels or kernels.index(k) >= len(names):
                continue
            if disp[k].index(int(r["Dispatch_Id"])) == 0:
                continue  # warm-up
            case = names[kernels.index(k)]
            c = per.setdefault(case, {})
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            c.setdefault(r["Counter_Name"], []).append((float(r["Counter_Value"]), dur))
    out = {}
    for case in names:
        e = dict(ev["shapes"][case])
        c = per.get(case, {})
        avg = {k: sum(v for v, _ in xs) / len(xs) for k, xs in c.items()}
        durs = [t for xs in c.values() for _, t in xs]
        row = {"events": e, "pmc_per_dispatch": {k: float(f"{v:.4e}") for k, v in sorted(avg.items())}}
        insts = avg.get("SQ_INSTS_VMEM_RD", 0.0) + avg.get("SQ_INSTS_VMEM_WR", 0.0)
        row["inst_kind"] = "vmem"
        if not insts and avg.get("SQ_INSTS_LDS"):
            insts, row["inst_kind"] = avg["SQ_INSTS_LDS"], "lds"
        if insts:
            per_inst = {}
            for k, lab in (("TD_TD_BUSY_sum", "td_busy_cycles_per_cu"), ("TA_TA_BUSY_sum", "ta_busy_cycles_per_cu"),
                           ("TD_TC_STALL_sum", "td_tc_stall_cycles_per_cu"),
                           ("TCP_TOTAL_CACHE_ACCESSES_sum", "tcp_accesses"),
                           ("TCP_TCC_READ_REQ_sum", "l2_read_reqs")):
                if k in avg:
                    # TD / TA busy summed over the CUs that ran the instructions: per CU and
                    # per instruction = sum / instructions (each instruction runs on one CU)
                    per_inst[lab] = round(avg[k] / insts, 3)
            row["per_vmem_inst"] = per_inst
            if avg.get("GRBM_GUI_ACTIVE") and durs:
                dur = sum(durs) / len(durs)
                clk = avg["GRBM_GUI_ACTIVE"] / N_XCD / dur
                row["clock_hz"] = float(f"{clk:.4e}")
                # CU cycles per instruction at saturation: the launch's cycles x CUs / instructions
                row["cu_cycles_per_inst"] = round(e["ms"] * 1e-3 * clk * ev["cus"] / insts, 3)
                if avg.get("TD_TD_BUSY_sum"):
                    row["td_busy_frac"] = round(avg["TD_TD_BUSY_sum"] / N_CU / (e["ms"] * 1e-3 * clk), 4)
        out[case] = row
    return out


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
    sh = shapes_summary(d)
    if sh:
        out["shapes"] = sh
    out["source"] = "tools/ubench.hip, tools/ubench_shapes.hip under rocprofv3 --pmc (tools/gpu_ubench.sh)"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
