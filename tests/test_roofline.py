"""bench.py's roofline on CPU: the data-return model and the
bound are reproducible from committed files alone.

* the per-shape costs come from profiles/ubench.json "shapes" (tools/ubench_shapes.hip
  under rocprofv3): a wave64 dwordx4 takes 16 TD processing cycles whatever its
  coherence, a scratch-shaped dword load / store far fewer;
* the committed C4 PMC entry and the bench line of the same build
  (profiles/r06/final/pmc_c4) give the model the bench line reports, and the model
  accounts for most of the PMC-measured processing (TD busy - TC stall);
* TD busy - an occupancy - is reported but never chosen as the bound once the model
  exists: the bound is the largest RATE fraction (VALU issue on C4).
"""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

FINAL = os.path.join(REPO, "profiles", "r06", "final", "pmc_c4")


def test_shape_costs_calibrated():
    c = bench.shape_costs()
    assert c is not None
    assert 15.5 <= c["x4"] <= 16.5 and 15.5 <= c["prim_x4"] <= 16.5
    # more distinct lines add waiting, not processing
    assert 15.5 <= c["x4_k64"] <= 16.5 and c["stall"]["x4_k64"] > 40
    assert 3.0 <= c["dword_load"] <= 5.0 and 1.0 <= c["dword_store"] <= 3.0
    sh = json.load(open(os.path.join(REPO, "profiles", "ubench.json")))["shapes"]
    # coherence and active lanes do not change a dwordx4's cost
    for case in ("node_k1_l2", "node_k2_l2", "node_k4_l2", "node_act1", "node_act32"):
        assert abs(sh[case]["per_vmem_inst"]["td_busy_cycles_per_cu"] - 16.0) < 0.5, case
    # every saturating shape reads TD busy near 1: an occupancy, not a rate
    assert all(0.9 < sh[k]["td_busy_frac"] < 1.01 for k in ("node_k1_l2", "node_k64_l2", "lane_dwords_store"))


def _line_and_entry():
    line = json.loads(open(os.path.join(FINAL, "bench_traced.json")).read().strip().splitlines()[-1])
    entry = json.load(open(os.path.join(FINAL, "entry.json")))
    return line, entry


def test_c4_model_reproducible_from_profiles():
    line, entry = _line_and_entry()
    assert line["build_id"] == entry["build_id"]
    sh = line["roofline"]["stats_shapes"]
    dc = [0] * 48
    for k, i in bench.DC_SHAPES.items():
        dc[i] = sh[k]
    dur = min(entry["duration_ns_per_pass"]) * 1e-9
    clk = entry["cache"]["GRBM_GUI_ACTIVE"] / bench.N_XCD / dur
    m = bench.data_return_model(entry, dc, 2048 // 8 * 2048 // 8 * 32, line["kernel_ms_avg"] / 1e3, clk)
    assert m is not None
    assert 0.25 < m["frac"] < 0.45  # processing share of the launch
    assert 0.75 < m["model_over_pmc_processing"] < 1.05
    assert m["pmc_td_busy_frac"] > 0.9 and m["pmc_tc_stall_frac"] > 0.45
    # the 7 dwordx4 of a vector node trip dominate what is processed
    assert max(m["parts_frac"], key=m["parts_frac"].get) == "node_loads"


def test_bound_is_a_rate_not_td_busy():
    line, entry = _line_and_entry()
    sh = line["roofline"]["stats_shapes"]
    dc = [0] * 48
    for k, i in bench.DC_SHAPES.items():
        dc[i] = sh[k]
    diag = {"rays_processed": line["rays_per_step"], "node_visits": 1, "leaf_visits": 1, "prim_tests": 1}
    r = bench.roofline(entry, line["kernel_ms_avg"] / 1e3, 1.0, diag, None, model_in=(dc, 2097152))
    assert r["ceilings"]["vmem_td"]["frac"] > r["ceilings"]["valu_issue"]["frac"]  # TD busy reads highest ...
    assert r["bound"] == "valu_issue"  # ... and is not the bound
    assert r["data_return_model"]["frac"] == pytest.approx(r["ceilings"]["vmem_model"]["frac"])


def test_ceilings_recomputed_from_committed_files():
    """tools/dr_model.py --ceilings: the shipped build's C4 bench line (with its
    roofline) and its PMC entry give back the line's bound and fraction."""
    import subprocess
    line = json.loads([x for x in open(os.path.join(REPO, "profiles", "r06", "final", "c4.json"))
                       if x.startswith("{")][-1])
    entry = os.path.join(FINAL, "entry.json")
    assert json.load(open(entry))["build_id"] == line["build_id"]
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "dr_model.py"), "--ceilings",
                          os.path.join(REPO, "profiles", "r06", "final", "c4.json"), entry],
                         capture_output=True, text=True, check=True).stdout
    r = json.loads(out)
    assert r["bound"] == line["roofline"]["bound"] == "valu_issue"
    assert r["frac"] == pytest.approx(line["roofline"]["frac"], abs=1e-3)
    assert r["data_return_model"]["frac"] == pytest.approx(line["roofline"]["data_return_model"]["frac"], abs=1e-3)
