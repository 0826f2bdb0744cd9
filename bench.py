#!/usr/bin/env python
"""bench.py — throughput of the HIP sampling loop on BASELINE.json's metric.

Workload (BASELINE.json configs[3]): scene 2 of scenes.zig
(bunny.obj + ground sphere, BVH), 2048x2048 pixels, 1024 samples per pixel,
max depth 20, counter RNG seeded 42.  One step = one full frame: every rank
renders its 8x8 tiles (tile t -> rank t % N) with the scene already resident
in HBM, the tiles are gathered to rank 0 over RCCL (torch.distributed "nccl")
and assembled into the reference's framebuffer layout
(zraytrace_amd.dist.TileFrame).  The frame is fixed as N grows: "scaling":
"strong".

value = rays of all ranks (raytrace.zig:69's rays_processed, counted on the
device) / the max-over-ranks wall time of the timed steps, in Mrays/s.

roofline: the render kernel's position against every ceiling it could be
bound by - TD (vector-memory data return) busy, VALU issue, L1 (TCP)
accesses, L1 -> L2 requests, HBM - each "achieved" = a per-launch PMC count
(rocprofv3 passes of this exact config, profiles/latest_pmc.json) / the
launch's HIP-event time measured in this run, against per-clock peaks measured
by tools/ubench.hip (profiles/ubench.json); "bound" is the ceiling with the
largest fraction.

Run: python bench.py [--gpus N --steps K --warmup W]
     N > 1, one process per GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
     N > 1, one process for all GPUs (no launcher, WORLD_SIZE unset): python bench.py --gpus N
       - zrt_multi_* over devices 0..N-1: one context per GPU, ncclCommInitAll
       communicators and one ncclGather per frame inside libzrt;
       --devices 0,0 rehearses it with two ranks on one GPU (device copies).
       Fewer than N visible GPUs is an error (exit 2), never a silent N=1 line.
"""
import argparse
import hashlib
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Mrays/s + achieved HBM GB/s, bunny BVH @ 2048², 1024spp, 1/2/4/8 GPUs"
SCENES = {0: "manAndBall: models/Man_LOD3.obj + ground sphere", 1: "threeBalls: 7 spheres",
          2: "bunnyAndBall: models/bunny.obj + ground sphere", 3: "teapotAndBall: models/teapot.obj + ground sphere",
          4: "teapotAndBallCircle: teapot + ring of spheres", 5: "goat: high_poly_goat.obj + ground sphere",
          6: "texturedTeapot: the C5 substitute, 1.6 M subdivided teapot triangles + image textures"}
# 0-5: scenes.zig:267-277; 6: DESIGN.md section 4

HBM_PEAK_GBS = 8000.0  # HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
N_CU, N_SIMD, N_XCD = 256, 1024, 8


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes(st, n_work_units, n_pixels):
    """Bytes the sampling loop must touch per launch:
    per node record read (32 B binary/reference node; 128 B wide node, which
    also carries its leaf children's boxes), 48 B per triangle test, 16 B per sphere test,
    64 B per shaded hit (16 B shade record + 48 B material), 4 B (8-bit store) or 12 B (f32) per texel,
    8 B per scatter (its 4-B attenuation code pushed + read back), 16 B per chunk sum
    written and read, 12 B per output pixel."""
    tri = st["prim_tests"] - st["sphere_tests"]
    return (st["node_bytes"] * st["node_visits"] + 48 * tri + 16 * st["sphere_tests"] + 64 * st["shade_fetches"]
            + (st["texel_bytes"] or 12) * st["texel_fetches"] + 8 * st["reflections"] + 32 * n_work_units + 12 * n_pixels)


def pmc_entry(config, build_id):
    """(entry, reason): the PMC record of render_kernel for this exact config AND
    this exact kernel build (profiles/latest_pmc.json, written by
    tools/make_latest_pmc.py from rocprofv3 --pmc passes, keyed by
    zrt_build_id()); (None, why) when there is none, so counters of another
    build are never attached to this one."""
    try:
        with open(os.path.join(REPO, "profiles", "latest_pmc.json")) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, "profiles/latest_pmc.json missing"
    stale = None
    for e in d.get("entries", []):
        if e.get("config") != config:
            continue
        if e.get("build_id") == build_id:
            return e, None
        stale = e.get("build_id")
    if stale is not None:
        return None, f"PMC entry for this config was taken on build {stale}, this library is {build_id}"
    return None, "no PMC entry for this config"


# The guide's architectural issue rate: one wave64 VALU instruction per 2 cycles
# per SIMD (MI355X_MICROARCH.md).  tools/ubench.hip's single-kernel measurement
# (profiles/ubench.json) reached 0.419 of a cycle, i.e. 84 % of it; the roofline
# prices against the architectural figure and reports the measured one beside it.
VALU_ISSUE_PER_SIMD_CLK = 0.5


def ubench_peaks():
    """Per-clock ceilings measured by tools/ubench.hip under rocprofv3 on the GPU box
    (profiles/ubench.json, tools/gpu_ubench.sh); the guide's figures where absent.
    VALU issue is always the guide's architectural rate (VALU_ISSUE_PER_SIMD_CLK)."""
    try:
        with open(os.path.join(REPO, "profiles", "ubench.json")) as f:
            p = dict(json.load(f)["peaks_per_clock"])
        src = "profiles/ubench.json (tools/ubench.hip, rocprofv3 --pmc)"
    except (OSError, ValueError, KeyError):
        p = {"tcp_accesses_per_cu": 1.0, "l2_read_req_per_cu": 0.375}
        src = "MI355X_MICROARCH.md (64 B/clk/CU L1; L2 34.5 TB/s)"
    p["valu_measured_per_simd"] = p.get("valu_insts_per_simd")
    p["valu_insts_per_simd"] = VALU_ISSUE_PER_SIMD_CLK
    return p, src + "; VALU issue: MI355X_MICROARCH.md, 0.5 wave64 inst/SIMD/clk"


# zrt_ctx_debug_counters slots of the STATS launch (render.hip kVNodeTrips ..):
# the FAST loops' vector-memory wave-instructions by shape
DC_SHAPES = {"vnode_trips": 32, "vnode_lines": 33, "snode_trips": 34, "rb_trips": 35, "vprim_trips": 36,
             "vprim_lines": 37, "sprim_trips": 38, "vshade_trips": 39, "att_w_trips": 40, "att_r_trips": 41,
             "vnode_cost": 42, "vprim_cost": 43}


def shape_costs():
    """TD (vector data return) cycles per wave-instruction of each load shape the
    render kernel issues, measured alone with the whole chip by
    tools/ubench_shapes.hip under rocprofv3 (profiles/ubench.json "shapes"), split
    into processing (TD_TD_BUSY - TD_TC_STALL) and waiting for the cache
    (TD_TC_STALL).  A wave64 dwordx4 load takes 16 processing cycles whether its
    lanes read 1, 2, 4 or 64 records and whether 1 or 64 lanes are active (more
    distinct lines add TC-stall cycles: one per line past 16); a dword per lane
    (256 B, the scratch layout) ~4.1 as a load, ~1.9 as a store (+ ~8.8 waiting
    for the write path).  None if the file has no shapes."""
    try:
        with open(os.path.join(REPO, "profiles", "ubench.json")) as f:
            sh = json.load(f)["shapes"]
    except (OSError, ValueError, KeyError):
        return None

    def proc(case):
        p = sh[case]["per_vmem_inst"]
        return round(p["td_busy_cycles_per_cu"] - p.get("td_tc_stall_cycles_per_cu", 0.0), 3)

    def stall(case):
        return sh[case]["per_vmem_inst"].get("td_tc_stall_cycles_per_cu")
    try:
        return {"x4": proc("node_k1_l2"), "x4_k64": proc("node_k64_l2"), "prim_x4": proc("prim_k1"),
                "dword_load": proc("lane_dwords_load"), "dword_store": proc("lane_dwords_store"),
                "stall": {"x4_k64": stall("node_k64_l2"), "dword_load": stall("lane_dwords_load"),
                          "dword_store": stall("lane_dwords_store")},
                "source": "profiles/ubench.json shapes (tools/ubench_shapes.hip, rocprofv3 --pmc): "
                          "TD_TD_BUSY - TD_TC_STALL per wave-instruction at saturation"}
    except KeyError:
        return None


def data_return_model(pmc, dc, n_units, kernel_s, clk):
    """The render launch's vector-memory data-return (TD) processing cycles,
    modelled (DESIGN.md §4 "The data-return model"): the STATS launch's wave-
    instruction counts per load shape (dc: zrt_ctx_debug_counters, DC_SHAPES) x
    each shape's calibrated processing cycles (shape_costs), plus the vector-memory
    instructions PMC counts beyond those - scratch (spilled registers' reloads and
    stores, one dword per lane) - at the dword costs.  frac = modelled processing
    cycles per CU / the launch's cycles: the share of the data-return path's
    calibrated throughput the launch uses.  Checked against the PMC pass: the
    model over (TD_TD_BUSY - TD_TC_STALL), and the cycles TD spent waiting for the
    cache (TD_TC_STALL) per launch cycle, reported beside it."""
    c = shape_costs()
    sq, cache = (pmc or {}).get("sq") or {}, (pmc or {}).get("cache") or {}
    if not c or not sq.get("SQ_INSTS_VMEM_RD") or dc is None or len(dc) <= max(DC_SHAPES.values()):
        return None
    n = {k: int(dc[i]) for k, i in DC_SHAPES.items()}
    if not n["vnode_trips"] and not n["snode_trips"]:
        return None  # not a FAST loop (or a library without the shape counters)
    rd_known = 7 * n["vnode_trips"] + n["rb_trips"] + 3 * n["vprim_trips"] + n["vshade_trips"] + n["att_r_trips"]
    wr_known = n["att_w_trips"] + n_units
    scratch_rd = max(0.0, sq["SQ_INSTS_VMEM_RD"] - rd_known)
    scratch_wr = max(0.0, sq.get("SQ_INSTS_VMEM_WR", 0.0) - wr_known)
    parts = {
        "node_loads": 7 * c["x4"] * n["vnode_trips"],  # 7 dwordx4 per vector node trip (the 8th: leaf_refs)
        "leaf_refs": c["x4"] * n["rb_trips"],
        "prim_loads": 3 * c["prim_x4"] * n["vprim_trips"],
        "shade_loads": c["x4"] * n["vshade_trips"],
        "att_rows": c["dword_store"] * n["att_w_trips"] + c["dword_load"] * n["att_r_trips"],
        "chunk_sums": c["x4"] * n_units,  # one dwordx4 store per unit
        "scratch_loads": c["dword_load"] * scratch_rd,
        "scratch_stores": c["dword_store"] * scratch_wr,
    }
    total = sum(parts.values())
    cyc = kernel_s * clk  # the launch's cycles per CU
    out = {"bound": "vmem_data_return", "processing_cycles_per_launch": float(f"{total:.4e}"),
           "frac": round(total / N_CU / cyc, 4),
           "parts_frac": {k: round(v / N_CU / cyc, 4) for k, v in parts.items()},
           "inputs": {**n, "n_units": int(n_units), "pmc_vmem_rd": sq["SQ_INSTS_VMEM_RD"],
                      "pmc_vmem_wr": sq.get("SQ_INSTS_VMEM_WR"), "scratch_rd_insts": scratch_rd,
                      "scratch_wr_insts": scratch_wr},
           "costs_td_processing_cycles_per_inst": c}
    busy, stall = cache.get("TD_TD_BUSY_sum"), cache.get("TD_TC_STALL_sum")
    if busy and stall is not None:
        out["pmc_processing_frac"] = round((busy - stall) / N_CU / cyc, 4)
        out["model_over_pmc_processing"] = round(total / (busy - stall), 4)
        out["pmc_tc_stall_frac"] = round(stall / N_CU / cyc, 4)
        out["pmc_td_busy_frac"] = round(busy / N_CU / cyc, 4)
        out["note"] = ("TD busy = processing (the model's rate against the calibrated 16 cycles per dwordx4) + "
                       "TC stall (TD waiting for the vector cache: L1 misses, the write path)")
    if cache.get("TCP_TCC_READ_REQ_sum") is not None:
        out["pmc_l2_read_reqs_per_vmem_rd"] = round(cache["TCP_TCC_READ_REQ_sum"] / sq["SQ_INSTS_VMEM_RD"], 3)
    return out


def roofline(pmc, kernel_s, algo_bytes, diag, pmc_reason=None, model_in=None):
    """The render launch against every ceiling it could be bound by.  Per ceiling:
    the PMC count per launch (rocprofv3 pass of this exact config) / the launch's
    HIP-event time measured in this run = achieved, against the measured per-clock
    peak x the clock the PMC pass saw (GRBM_GUI_ACTIVE per XCD / its duration):
      vmem_td     TD (vector-memory data return) busy cycles per CU; peak = every cycle
      valu_issue  wave64 VALU instructions; peak = the 2-source class issue rate
      l1_access   TCP (L1) cache accesses; peak = the best load pattern's rate
      l2_lines    L1 -> L2 read requests; peak = an all-miss L1 pattern's rate
      hbm         (2 FETCH_SIZE + WRITE_SIZE) KiB; peak = 8 TB/s
      vmem_model  modelled data-return cycles per CU (data_return_model: the STATS
                  launch's wave-instructions per load shape x their ubench_shapes
                  costs); peak = every cycle of the launch
    bound = the rate ceiling with the largest fraction; the TD busy
    counter is reported beside the model, not chosen, when the model exists."""
    out = {"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None,
           "kernel_s": round(kernel_s, 6)}
    if not pmc:
        out["reason"] = pmc_reason
    rows = {}
    if pmc:
        peaks, src = ubench_peaks()
        sq, cache = pmc.get("sq") or {}, pmc.get("cache") or {}
        dur = min(pmc["duration_ns_per_pass"]) * 1e-9
        clk = cache["GRBM_GUI_ACTIVE"] / N_XCD / dur if cache.get("GRBM_GUI_ACTIVE") else 2.4e9
        out["clock_ghz"] = round(clk / 1e9, 3)
        spec = {"vmem_td": (cache.get("TD_TD_BUSY_sum", 0) / N_CU or None, clk, "TD busy cycles/s per CU"),
                "valu_issue": (sq.get("SQ_INSTS_VALU"), peaks["valu_insts_per_simd"] * N_SIMD * clk,
                               "wave64 VALU inst/s"),
                "l1_access": (cache.get("TCP_TOTAL_CACHE_ACCESSES_sum"), peaks["tcp_accesses_per_cu"] * N_CU * clk,
                              "TCP accesses/s"),
                "l2_lines": (cache.get("TCP_TCC_READ_REQ_sum"), peaks["l2_read_req_per_cu"] * N_CU * clk,
                             "L1->L2 read requests/s"),
                "hbm": (pmc.get("hbm_bytes_per_launch"), HBM_PEAK_GBS * 1e9, "B/s")}
        for k, (per_launch, peak, unit) in spec.items():
            if not per_launch:
                continue
            a = per_launch / kernel_s
            rows[k] = {"per_launch": per_launch, "achieved": float(f"{a:.4e}"), "peak": float(f"{peak:.4e}"),
                       "unit": unit, "frac": round(a / peak, 4)}
        out["peak_source"] = src
        out["traffic"] = pmc.get("hbm_bytes_per_launch")
        out["pmc_source"] = pmc.get("source")
        out["valu_lane_util"] = sq.get("valu_lane_util")
        out["pmc_build_id"] = pmc.get("build_id")
        if cache.get("TCC_HIT_sum") is not None and cache.get("TCC_MISS_sum"):
            out["l2_hit_frac"] = round(cache["TCC_HIT_sum"] / (cache["TCC_HIT_sum"] + cache["TCC_MISS_sum"]), 4)
    if pmc and model_in is not None:
        m = data_return_model(pmc, model_in[0], model_in[1], kernel_s, clk)
        if m:
            out["data_return_model"] = m
            rows["vmem_model"] = {"per_launch": m["processing_cycles_per_launch"],
                                  "achieved": float(f"{m['processing_cycles_per_launch'] / N_CU / kernel_s:.4e}"),
                                  "peak": float(f"{clk:.4e}"), "unit": "modelled TD processing cycles/s per CU",
                                  "frac": m["frac"]}
    if rows:
        # TD_TD_BUSY counts cycles TD is processing OR waiting for data: a utilisation,
        # not a rate (ubench_shapes: ~0.98 at every saturating shape), so where the
        # data-return model exists the bound is chosen among the rates
        cand = [k for k in rows if not (k == "vmem_td" and "vmem_model" in rows)]
        b = max(cand, key=lambda k: rows[k]["frac"])
        out.update({"bound": b, "achieved": rows[b]["achieved"], "peak": rows[b]["peak"], "unit": rows[b]["unit"],
                    "frac": rows[b]["frac"]})
        if "valu_issue" in rows and out.get("valu_lane_util"):
            # issue fraction x active-lane fraction: the share of the chip's VALU lane slots doing work
            rows["valu_issue"]["useful_lane_frac"] = round(rows["valu_issue"]["frac"] * out["valu_lane_util"], 4)
            rows["valu_issue"]["measured_peak_per_simd_clk"] = peaks.get("valu_measured_per_simd")
        if "hbm" in rows:
            out["hbm_gbs_measured"] = round(rows["hbm"]["achieved"] / 1e9, 1)
            out["hbm_frac"] = rows["hbm"]["frac"]
    out["ceilings"] = rows
    rays = max(1, diag["rays_processed"])
    out["algorithmic"] = {
        "bytes_per_launch": int(algo_bytes), "gbs": round(algo_bytes / kernel_s / 1e9, 1),
        "note": "bytes each ray's node/primitive/material reads and path-state writes touch; served by LDS/L1/L2 "
                "(the bunny scene is ~2 MB), so this is not an HBM figure and carries no HBM fraction",
        "per_ray": {"node_visits": round(diag["node_visits"] / rays, 2),
                    "leaf_visits": round(diag["leaf_visits"] / rays, 2),
                    "prim_tests": round(diag["prim_tests"] / rays, 2),
                    "bytes": round(algo_bytes / rays, 1)}}
    return out


def n1_frame_hash(config):
    """The committed frame hash of this config rendered on ONE GPU
    (profiles/frame_hashes.json); an N-rank frame must equal it bit for bit
    (the image is independent of the partition).  None if absent."""
    try:
        with open(os.path.join(REPO, "profiles", "frame_hashes.json")) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    for e in d.get("entries", []):
        if e.get("config") == config:
            return e.get("frame_sha1")
    return None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(scene, scene_index, depth, target_s=15.0):
    """The oracle (single-threaded C restatement, reference RNG stream) on a
    bounded sample of the same scene at the bench's depth: 128x128 pixels (16x16
    for a mesh of > 100k primitives, whose reference loose slab test visits most of
    the tree per ray), one probe sample per pixel, then as many samples per pixel
    as fill about `target_s` seconds of one core.  Also config C1 in full (scene
    1, 256x256 @ 16 spp, depth 30: BASELINE.md section 3)."""
    import zraytrace_amd as z
    from oracle import oracle_py as O
    big = scene.view.contents.n_prims > 100_000
    w = h = 16 if big else 128
    p = z.RenderParams(w, h, 1, depth, rng_mode=z.ZRT_RNG_REFERENCE_STREAM)
    _, st = O.render(scene.view, scene.camera, p)
    probe_s = st["render_ms"] / 1e3
    spp = 1
    if probe_s < target_s / 2:
        spp = max(1, min(4096, int(target_s / max(probe_s, 1e-4))))
        p = z.RenderParams(w, h, spp, depth, rng_mode=z.ZRT_RNG_REFERENCE_STREAM)
        _, st = O.render(scene.view, scene.camera, p)
    dt = st["render_ms"] / 1e3  # the sampling loop only; its BVH build is timed apart (raytrace.zig:150)
    s1 = z.load_scene(1)
    _, c1 = O.render(s1.view, s1.camera, z.RenderParams(256, 256, 16, 30, rng_mode=z.ZRT_RNG_REFERENCE_STREAM))
    c1_s = c1["render_ms"] / 1e3
    return {"value": st["rays_processed"] / dt / 1e6, "unit": "Mrays/s", "cores": 1, "kind": "port",
            "sample": f"oracle/ (C restatement of the Zig path, reference RNG stream), scene {scene_index} "
                      f"({SCENES[scene_index].split(':')[0]}), {w}x{h} @ {spp} spp, depth {depth}: "
                      f"{st['rays_processed']} rays in {dt:.2f} s on 1 core (BVH build "
                      f"{st['preprocess_ms'] / 1e3:.2f} s excluded)",
            "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            # the one-core rate scaled linearly to every core of the box - an upper
            # bound for the single-threaded reference (it has no threads), labelled as such
            "all_cores_linear": {"value": round(st["rays_processed"] / dt / 1e6 * (os.cpu_count() or 1), 3),
                                 "unit": "Mrays/s", "cores": os.cpu_count(),
                                 "note": "linear extrapolation of the 1-core figure (not measured; the reference "
                                         "is single-threaded)"},
            "c1_full": {"config": "scene 1 (7 spheres, list), 256x256 @ 16 spp, depth 30, reference RNG stream",
                        "rays": c1["rays_processed"], "seconds": round(c1_s, 3),
                        "mrays_per_s": round(c1["rays_processed"] / c1_s / 1e6, 3), "cores": 1}}


def reference_check(frame_obj, params, fast_sha1, z):
    """One untimed launch of the same frame with the REFERENCE traversal (the
    reference's left-first DFS and loose slab test, bvh.zig:187-205): its rate
    separates the algorithm from the hardware, and its frame must hash equal to
    FAST's (the exactness claim of DESIGN.md §3 at the full bench size)."""
    pref = z.RenderParams(**{**params.__dict__, "traversal": z.ZRT_TRAVERSAL_REFERENCE})
    t = time.perf_counter()
    kms = frame_obj.step(pref)
    st = frame_obj.ctx.stats()
    img = frame_obj.image()
    wall = time.perf_counter() - t
    sha = hashlib.sha1(img.tobytes()).hexdigest()
    return {"traversal": "reference", "mrays_per_s": round(st["rays_processed"] / (st["render_ms"] / 1e3) / 1e6, 2),
            "kernel_ms": round(kms, 2), "render_ms": round(st["render_ms"], 2), "wall_s": round(wall, 2),
            "rays": st["rays_processed"], "frame_sha1": sha, "frame_equal_to_fast": sha == fast_sha1}


def fail(msg, code=2):
    log(f"bench.py: error: {msg}")
    sys.exit(code)


def main_multi(args, devices):
    """--gpus N without a launcher: every GPU driven from this one process through
    zrt_multi_* (per-device contexts, ncclCommInitAll, one ncclGather to
    devices[0] and the assemble there).  A step = one zrt_multi_render: every
    rank's launch enqueued, then the gather and assemble, synchronous; the frame
    stays in devices[0]'s HBM (no PCIe copy in the timed region)."""
    import torch
    n_vis = torch.cuda.device_count()  # (counts without initialising a device)
    if n_vis == 0 or max(devices) >= n_vis:
        fail(f"--gpus {args.gpus} needs devices {sorted(set(devices))}, {n_vis} visible")
    import zraytrace_amd as z
    from zraytrace_amd.dist import tile_counts
    scene = z.load_scene(args.scene)
    trav = {"fast": z.ZRT_TRAVERSAL_FAST, "reference": z.ZRT_TRAVERSAL_REFERENCE,
            "binary": z.ZRT_TRAVERSAL_BINARY}[args.traversal]
    params = z.RenderParams(args.width, args.height, args.spp, args.depth, traversal=trav,
                            sample_chunk=args.chunk)
    m = z.MultiContext(scene, params, devices)
    distinct = sorted(set(devices))
    for i in range(args.warmup):
        t = time.perf_counter()
        m.render(scene.camera, params, copy_out=False)
        log(f"[multi] warmup {i + 1}/{args.warmup}: {time.perf_counter() - t:.2f} s")
    for d in distinct:
        torch.cuda.synchronize(d)
    rank_ms, gather_ms = [], []
    t0 = time.perf_counter()
    for i in range(args.steps):
        _, st = m.render(scene.camera, params, copy_out=False)
        rank_ms.append(m.rank_ms())
        gather_ms.append(st["gather_ms"])
        log(f"[multi] step {i + 1}/{args.steps}: slowest rank kernel {max(rank_ms[-1]):.1f} ms, "
            f"gather+assemble {gather_ms[-1]:.2f} ms")
    for d in distinct:
        torch.cuda.synchronize(d)
    elapsed = time.perf_counter() - t0
    frame_sha1 = hashlib.sha1(m.frame().tobytes()).hexdigest()
    _, diag = m.render(scene.camera, z.RenderParams(**{**params.__dict__, "flags": params.flags | z.ZRT_FLAG_STATS}),
                       copy_out=False)
    assert diag["rays_processed"] == st["rays_processed"], "diagnostic launch diverged"
    m.close()

    n = len(devices)
    chunk = args.chunk or 32  # ZRT_DEFAULT_SAMPLE_CHUNK
    counts = tile_counts(z.RenderParams(**{**params.__dict__, "world_size": n}))
    n_units = sum(counts) * ((args.spp + chunk - 1) // chunk)
    per_rank = [sum(r[k] for r in rank_ms) / len(rank_ms) for k in range(n)]
    slowest_s = max(per_rank) / 1e3
    algo = algorithmic_bytes(diag, n_units, diag["pixels_processed"])
    # the ceilings are priced from PMC passes at N=1 only; here the frame's
    # algorithmic bytes spread over the ranks against the slowest rank's kernel
    roof = {"bound": None, "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None,
            "reason": "PMC passes are taken at N=1 only", "kernel_s": round(slowest_s, 6),
            "algorithmic": {"bytes_per_launch": int(algo), "gbs_per_gpu": round(algo / n / slowest_s / 1e9, 1),
                            "per_ray": {"node_visits": round(diag["node_visits"] / max(1, diag["rays_processed"]), 2),
                                        "bytes": round(algo / max(1, diag["rays_processed"]), 1)}}}
    key = {"scene": args.scene, "width": args.width, "height": args.height, "spp": args.spp,
           "max_depth": args.depth, "traversal": args.traversal, "sample_chunk": chunk}
    ref_hash = n1_frame_hash(key)
    out = {
        "metric": METRIC,
        "value": round(st["rays_processed"] * args.steps / elapsed / 1e6, 2),
        "unit": "Mrays/s",
        "n_gpus": len(distinct),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic: the reference's own scene {args.scene} ({SCENES[args.scene]}), no dataset",
        "config": {"workload": f"scene {args.scene} ({SCENES[args.scene].split(':')[0]}) "
                               f"{'BVH' if st['used_bvh'] else 'list'}, {args.width}x{args.height} @ "
                               f"{args.spp} spp, max depth {args.depth}",
                   "scene": args.scene, "width": args.width, "height": args.height, "spp": args.spp,
                   "max_depth": args.depth, "traversal": args.traversal, "sample_chunk": chunk,
                   "rng": "counter (Xoroshiro128+ per pixel-sample, seed 42)",
                   "parallelism": f"image tiles 8x8 round-robin over {n} rank(s) on devices {devices}, "
                                  f"one process (zrt_multi_*), "
                                  + ("ncclGather over xGMI" if len(distinct) == n and n > 1
                                     else "device-to-device copies (ranks share a GPU)")},
        "launcher": "none (one process, zrt_multi_*)",
        "ranks": n,
        "devices": devices,
        "rays_per_step": int(st["rays_processed"]),
        "samples_per_step": int(st["samples_processed"]),
        "rays_per_sample": round(st["rays_processed"] / max(1, st["samples_processed"]), 4),
        "kernel_ms_slowest_rank": round(max(per_rank), 2),
        "roofline": roof,
        "parity": "bit-exact vs oracle (tests/test_gpu_parity.py); frame vs the committed N=1 frame below",
        "frame_sha1": frame_sha1,
        "frame_sha1_n1": ref_hash,
        "frame_equal_to_n1": (frame_sha1 == ref_hash) if ref_hash else None,
        "build_id": z.build_id(),
        "abi_version": z.lib().zrt_abi_version(),
        "per_rank_ms": {"kernel": [round(x, 3) for x in per_rank],
                        "gather_assemble": round(sum(gather_ms) / len(gather_ms), 3)},
    }
    if len(distinct) < n:
        out["scaling_note"] = (f"{n} ranks share {len(distinct)} GPU(s): value rehearses the N-rank path (launches, "
                               "gather, assemble, frame equality) and is not a scaling figure; the ranks' kernels "
                               "run concurrently on the same CUs, so per_rank_ms.kernel is each rank's share of "
                               "one GPU, not its time alone")
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", type=int, default=2)
    ap.add_argument("--width", type=int, default=2048)
    ap.add_argument("--height", type=int, default=2048)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--depth", type=int, default=20)
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--traversal", choices=["fast", "reference", "binary"], default="fast")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--guard", action="store_true",
                    help="render with ZRT_FLAG_GUARD (the grazing-triangle guard; the path-pool loop carries it)")
    ap.add_argument("--no-reference-check", action="store_true",
                    help="skip the untimed REFERENCE-traversal launch of the same frame (N=1 only)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (RCCL, one GPU per rank) or gloo (rehearsal: ranks may share a GPU)")
    ap.add_argument("--device", type=int, default=None, help="GPU index (default: LOCAL_RANK)")
    ap.add_argument("--devices", default=None,
                    help="one-process path: comma-separated device per rank (e.g. 0,0 rehearses 2 ranks on GPU 0)")
    args = ap.parse_args()
    if args.gpus < 1:
        fail("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.devices):
        devices = [int(x) for x in args.devices.split(",")] if args.devices else list(range(args.gpus))
        if len(devices) < 1 or min(devices) < 0:
            fail(f"--devices {args.devices}: need one non-negative device index per rank")
        if not args.devices and len(devices) != args.gpus:
            fail(f"--gpus {args.gpus} does not match {len(devices)} devices")
        return main_multi(args, devices)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        fail(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if args.dist_backend == "nccl" and args.device is None:
        n_vis = torch.cuda.device_count()
        if local >= n_vis:
            fail(f"rank {rank} needs GPU {local}, {n_vis} visible")
    if args.device is not None:
        local = args.device
    torch.cuda.set_device(local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)

    import zraytrace_amd as z
    from zraytrace_amd.dist import TileFrame
    scene = z.load_scene(args.scene)
    trav = {"fast": z.ZRT_TRAVERSAL_FAST, "reference": z.ZRT_TRAVERSAL_REFERENCE,
            "binary": z.ZRT_TRAVERSAL_BINARY}[args.traversal]
    params = z.RenderParams(args.width, args.height, args.spp, args.depth, traversal=trav,
                            rank=rank, world_size=world, device=local, sample_chunk=args.chunk,
                            flags=z.ZRT_FLAG_GUARD if args.guard else 0)
    fr = TileFrame(scene, params, rank, world)

    for i in range(args.warmup):
        t = time.perf_counter()
        fr.step()
        torch.cuda.synchronize()
        log(f"[rank {rank}] warmup {i + 1}/{args.warmup}: {time.perf_counter() - t:.2f} s")

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_ms = []
    for i in range(args.steps):
        kernel_ms.append(fr.step())
        log(f"[rank {rank}] step {i + 1}/{args.steps}: kernel {kernel_ms[-1]:.1f} ms")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    st = fr.ctx.stats()  # Progress counters of the last timed launch (identical every step)
    # per-rank kernel and gather times of the timed steps (HIP events on the frame's stream)
    # (gather_ms holds the timed steps' gathers; None rather than a fake 0 if it has none)
    my_times = [sum(kernel_ms) / len(kernel_ms),
                sum(fr.gather_ms) / len(fr.gather_ms) if fr.gather_ms else float("nan")]
    frame_sha1 = hashlib.sha1(fr.image().tobytes()).hexdigest() if rank == 0 else None
    # Traffic diagnostics (node visits, primitive tests, ...) come from one extra,
    # untimed launch of the diagnostic kernel flavour: same traversal, same image.
    diag_kernel_ms = fr.step(z.RenderParams(**{**params.__dict__, "flags": params.flags | z.ZRT_FLAG_STATS}))
    diag = fr.ctx.stats()
    assert diag["rays_processed"] == st["rays_processed"], "diagnostic launch diverged"
    red = "cuda" if args.dist_backend == "nccl" else "cpu"
    rays = torch.tensor([float(st["rays_processed"]), float(st["samples_processed"])], dtype=torch.float64,
                        device=red)
    el = torch.tensor([elapsed], dtype=torch.float64, device=red)
    if world > 1:
        dist.all_reduce(rays, op=dist.ReduceOp.SUM)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    total_rays, total_samples = rays.tolist()
    elapsed = el.item()
    per_rank = [my_times]
    if world > 1:
        tt = torch.tensor(my_times, dtype=torch.float64, device=red)
        allt = [torch.zeros_like(tt) for _ in range(world)]
        dist.all_gather(allt, tt)
        per_rank = [x.tolist() for x in allt]

    if rank == 0:
        value = total_rays * args.steps / elapsed / 1e6
        avg_kernel_s = sum(kernel_ms) / len(kernel_ms) / 1e3
        chunk = args.chunk or 32  # ZRT_DEFAULT_SAMPLE_CHUNK
        n_units = fr.counts[rank] * ((args.spp + chunk - 1) // chunk)
        algo = algorithmic_bytes(diag, n_units, diag["pixels_processed"])
        pmc_key = {"scene": args.scene, "width": args.width, "height": args.height, "spp": args.spp,
                   "max_depth": args.depth, "traversal": args.traversal, "sample_chunk": chunk}
        bid = z.build_id()
        if world == 1:
            pe, why = pmc_entry(pmc_key, bid)
        else:
            pe, why = None, "PMC passes are taken at N=1 only"
        if bid.split("-")[0] != z.build_id_of_sources():
            pe, why = None, f"libzrt.so ({bid}) is stale against its sources ({z.build_id_of_sources()})"
        dc = fr.ctx.debug_counters(48)  # the STATS launch's counters (shapes, SIMD efficiency, writes)
        roof = roofline(pe, avg_kernel_s, algo, diag, why, model_in=(dc, n_units))
        # what the render launch writes to memory: each work unit's
        # 64 chunk sums (float4), the attenuation rows past the LDS ones (float4; STATS
        # counter kAttWrites of the diagnostic launch) and, on deep trees, the traversal
        # stack entries past the LDS rows (u32; kStackOvfWrites)
        wb = {"chunk_sums_B": 16 * 64 * n_units, "att_rows_B": 4 * int(dc[28]),  # 4-B att codes
              "stack_rows_B": 4 * int(dc[30])}  # FAST stack entries past the LDS rows (kStackOvfWrites)
        wb["payload_B"] = wb["chunk_sums_B"] + wb["att_rows_B"] + wb["stack_rows_B"]
        # what memory sees: a chunk-sum store is 1 KiB of whole lines; a row or stack
        # store is 4 B, and where the wave's lanes store to unrelated paths (every loop
        # but lockstep, whose lanes push the same row together) each is written back as
        # a 32-B sector of its own (L2 keeps no line long enough to merge a path's pushes
        # under the C5 fetch stream: profiles/r04/r04o, path-major rows)
        loop_id = int(st.get("sampling_loop", -1))
        granule = 4 if loop_id == 3 else 32
        wb["row_store_granule_B"] = granule
        wb["predicted_B"] = wb["chunk_sums_B"] + (granule // 4) * (wb["att_rows_B"] + wb["stack_rows_B"])
        if pe and pe.get("write_size_kb"):
            wb["pmc_write_B"] = int(pe["write_size_kb"] * 1024)
            wb["predicted_over_pmc"] = round(wb["predicted_B"] / wb["pmc_write_B"], 3)
            c = pe.get("cache") or {}
            if c.get("TCC_EA0_WRREQ_sum"):
                # L2 -> memory write requests: 64-B (whole line) and 32-B (partial) ones;
                # WRITE_SIZE = 64 x WRREQ_64B + 32 x the rest on gfx950
                n64 = c.get("TCC_EA0_WRREQ_64B_sum", 0.0)
                n32 = c["TCC_EA0_WRREQ_sum"] - n64
                wb["pmc_wrreq_64B"] = int(n64)
                wb["pmc_wrreq_32B"] = int(n32)
                wb["pmc_wrreq_bytes"] = int(64 * n64 + 32 * n32)
        roof["write_budget"] = wb
        # the STATS launch's vector-load shape counts (data_return_model's inputs), kept in
        # the line so the model can be recomputed against any PMC entry (tools/dr_model.py)
        roof["stats_shapes"] = {k: int(dc[i]) for k, i in DC_SHAPES.items()} if len(dc) > 43 else None
        if pe and pe.get("fetch_size_kb") is not None:
            # HBM bytes the sampling loop needs, apart from what spilled registers cost:
            # the measured reads (2 x FETCH_SIZE KiB, MI355X_MICROARCH.md's gfx950
            # correction) plus the predicted payload writes (chunk sums, global att and
            # stack rows at the store granule), never the scratch lines of spills
            useful = 2 * pe["fetch_size_kb"] * 1024 + wb["predicted_B"]
            roof["useful_hbm"] = {"bytes_per_launch": int(useful),
                                  "gbs": round(useful / avg_kernel_s / 1e9, 1),
                                  "frac": round(useful / avg_kernel_s / (HBM_PEAK_GBS * 1e9), 4),
                                  "note": "2 FETCH_SIZE (PMC) + predicted payload writes; hbm_frac also counts "
                                          "spill scratch lines written back (WRITE_SIZE)"}
        # SIMD efficiency of the loop (STATS launch, zrt_ctx_debug_counters slots 4 / 21-23):
        # lane node visits / (64 x the wave's traversal trips), and the lanes that ran a
        # rayColor step / (64 x loop iterations that ran one)
        loops = {0: "list", 1: "binary", 2: "reference", 3: "lockstep", 4: "wavefront", 5: "path pool",
                 6: "list, per-lane items"}
        # (an A/B variant built before zrt_stats.sampling_loop existed leaves it zero: "unknown", not "list")
        simd = {"sampling_loop": loops.get(int(st.get("sampling_loop", -1)), "unknown") if bid != "unknown"
                else "unknown"}
        if int(dc[21]):
            simd["traversal_lane_eff"] = round(int(dc[4]) / (64.0 * int(dc[21])), 4)
        if int(dc[22]):
            # (the path pool's lanes own two paths each and may shade both in one
            # loop iteration: there the ratio runs up to 2)
            simd["shade_lane_eff"] = round(int(dc[23]) / (64.0 * int(dc[22])), 4)
        roof["kernel"] = f"render_kernel (BVH {args.traversal} traversal)"
        roof["counters_from"] = f"one untimed ZRT_FLAG_STATS launch (kernel {diag_kernel_ms:.1f} ms)"
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: the reference's own scene {args.scene} ({SCENES[args.scene]}), no dataset",
            "config": {"workload": f"scene {args.scene} ({SCENES[args.scene].split(':')[0]}) "
                                   f"{'BVH' if st['used_bvh'] else 'list'}, {args.width}x{args.height} @ "
                                   f"{args.spp} spp, max depth {args.depth}",
                       "scene": args.scene, "width": args.width, "height": args.height, "spp": args.spp,
                       "max_depth": args.depth, "traversal": args.traversal, "sample_chunk": chunk,
                       "rng": "counter (Xoroshiro128+ per pixel-sample, seed 42)",
                       "grazing_guard": bool(args.guard),
                       "parallelism": f"image tiles 8x8 round-robin over {world} GPU(s) + RCCL gather"},
            "rays_per_step": int(total_rays),
            "samples_per_step": int(total_samples),
            "rays_per_sample": round(total_rays / max(1.0, total_samples), 4),
            "kernel_ms_avg": round(avg_kernel_s * 1e3, 2),
            "order_replays": diag["order_replays"],
            "simd": simd,
            "roofline": roof,
            "accel": {"reference_bvh_nodes": diag["bvh_nodes"], "reference_bvh_depth": diag["bvh_max_depth"],
                      "wide_nodes": diag["wide_nodes"], "node_bytes": diag["node_bytes"]},
            "parity": "bit-exact vs oracle (tests/test_gpu_parity.py)",
            "frame_sha1": frame_sha1,
            "build_id": bid,
            "abi_version": z.lib().zrt_abi_version(),
            "per_rank_ms": {"kernel": [round(x[0], 3) for x in per_rank],
                            "gather": [round(x[1], 3) if x[1] == x[1] else None for x in per_rank]},
        }
        ref_hash = n1_frame_hash(pmc_key)
        out["frame_sha1_n1"] = ref_hash
        out["frame_equal_to_n1"] = (frame_sha1 == ref_hash) if ref_hash else None
        if world == 1 and args.traversal == "fast" and st["used_bvh"] and not args.no_reference_check:
            if scene.n_prims <= 100_000:
                log("[rank 0] reference-traversal launch of the same frame ...")
                out["reference_traversal"] = reference_check(fr, params, frame_sha1, z)
            else:  # the reference's loose test visits most of a million-triangle tree per ray
                out["reference_traversal"] = {"skipped": f"{scene.n_prims} primitives: the reference's loose slab "
                                                         "test visits most of the tree per ray (hours per frame)"}
        if world == 1 and not args.no_cpu_baseline:
            log("[rank 0] cpu baseline (oracle, 1 core) ...")
            out["cpu_baseline"] = cpu_baseline(scene, args.scene, args.depth)
        print(json.dumps(out), flush=True)

    fr.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
