"""The N>1 plumbing on CPU: world-size-2 (and 3) gloo process groups.

Each rank fills its padded tile buffer with values that encode (rank, local
pixel index); rank 0 gathers with zraytrace_amd.dist.gather_tiles and scatters
the rank-major result with a numpy restatement of assemble_kernel's mapping.
Every pixel of the rendered area must come from the tile owner the partition
rule names (tile t -> rank t % world) and nothing may be lost or duplicated.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import zraytrace_amd as z
from zraytrace_amd.dist import gather_tiles, tile_counts


def assemble_numpy(gathered, counts, width, height, world):
    """Restatement of assemble_kernel's padded mode (render.hip) for the test:
    rank r's tiles start at tile r * max(counts); tiles past a rank's count are padding."""
    xbound = height                      # raytrace.zig:168
    tiles_x = (xbound + 7) // 8
    n_tiles = tiles_x * ((height + 7) // 8)
    stride = max(counts) * 64
    frame = np.zeros((height, width, 3), np.float32)
    owner = np.full((height, width), -1, np.int64)
    for i in range(world * stride):
        r, w = divmod(i, stride)
        lt, p = divmod(w, 64)
        t = lt * world + r
        if t >= n_tiles:
            assert lt >= counts[r], "a rank's own tile treated as padding"
            continue
        px = (t % tiles_x) * 8 + p % 8
        py = (t // tiles_x) * 8 + p // 8
        if px < xbound and py < height:
            assert owner[py, px] == -1, "pixel assembled twice"
            owner[py, px] = r
            frame[py, px] = gathered[i]
    return frame, owner


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, width, height, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = z.RenderParams(width, height, 4, 5, rank=rank, world_size=world)
        counts = tile_counts(p)
        n = max(counts) * 64
        tiles = torch.full((n * 3,), -1.0)
        local = torch.arange(counts[rank] * 64, dtype=torch.float32)
        v = torch.stack([torch.full_like(local, rank), local, local * 0 + 7], 1).reshape(-1)
        tiles[: v.numel()] = v
        g = gather_tiles(tiles, counts, rank, world, dst=0)
        if rank == 0:
            q.put((counts, g.numpy().reshape(-1, 3)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,width,height", [(2, 40, 40), (3, 37, 21)])
def test_gloo_gather_and_assemble(world, width, height):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, width, height, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    counts, gathered = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert len(gathered) == world * max(counts) * 64
    frame, owner = assemble_numpy(gathered, counts, width, height, world)
    xb = height
    assert (owner[:, :xb] >= 0).all() and (owner[:, xb:] == -1).all()
    assert (frame[:, :xb, 2] == 7).all()            # every rendered pixel came from a real tile slot
    tiles_x = (xb + 7) // 8
    ty, tx = np.mgrid[0:height, 0:xb] // 8
    assert (owner[:, :xb] == (ty * tiles_x + tx) % world).all()   # tile t -> rank t % world


def test_tile_counts_partition():
    for world in (1, 2, 4, 8):
        p = z.RenderParams(2048, 2048, 1, 1, world_size=world)
        c = tile_counts(p)
        assert sum(c) == 256 * 256 and max(c) - min(c) <= 1
