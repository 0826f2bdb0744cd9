"""SIMD efficiency of the FAST kernel per config (STATS flavour counters,
zrt_ctx_debug_counters slots 21-23): traversal lane efficiency = lane node
visits / (64 x wave traversal trips), step efficiency = lane rayColor steps /
(64 x wave loop iterations with a runnable lane).  GPU box only.
usage: python tools/simd_eff.py scene:W:H:SPP [...]  -> one JSON line per config"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import zraytrace_amd as z  # noqa: E402

def ctx_units(ctx, p):
    """Work units (tile x sample chunk) of the launch: each writes 64 chunk sums of 16 B."""
    chunk = p.sample_chunk or 32
    return ctx.tile_count(p) * ((p.samples_per_pixel + chunk - 1) // chunk)


for spec in sys.argv[1:] or ["2:2048:2048:16", "3:1024:1024:16", "6:4096:4096:4"]:
    sc, w, h, spp = (int(v) for v in spec.split(":"))
    s = z.load_scene(sc)
    depth = 30 if sc == 1 else 20
    p = z.RenderParams(w, h, spp, depth, flags=z.ZRT_FLAG_STATS | z.ZRT_FLAG_NO_SCHEDULE)
    ctx = z.RenderContext(s, p)
    buf = torch.zeros(ctx.tile_count(p) * 64 * 3, dtype=torch.float32, device="cuda")
    ctx.render_tiles(s.camera, p, buf.data_ptr())
    st = ctx.stats()
    c = ctx.debug_counters(32)
    trips, loops, lsteps = c[21], c[22], c[23]
    out = {"scene": sc, "width": w, "height": h, "spp": spp, "rays": st["rays_processed"],
           "node_visits": st["node_visits"], "trav_trips": trips, "loop_trips": loops, "lane_steps": lsteps,
           "trav_lane_eff": round(st["node_visits"] / max(1, 64 * trips), 4),
           "step_lane_eff": round(lsteps / max(1, 64 * loops), 4),
           "nodes_per_ray": round(st["node_visits"] / st["rays_processed"], 3),
           "trips_per_loop": round(trips / max(1, loops), 3), "kernel_ms": st["render_ms"],
           "global_nodes_per_ray": round(c[24] / st["rays_processed"], 3),
           "uniform_node_frac": round(c[25] / max(1, c[24]), 4),
           "prim_tests_per_ray": round(c[26] / st["rays_processed"], 3),
           "uniform_prim_frac": round(c[27] / max(1, c[26]), 4),
           "att_global_writes": c[28], "att_global_reads": c[29], "units": ctx_units(ctx, p),
           "chunk_sum_bytes": 16 * 64 * ctx_units(ctx, p)}
    print(json.dumps(out), flush=True)
    ctx.close()
