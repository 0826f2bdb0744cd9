"""Multi-GPU plumbing for the tile partition.

8x8 tiles are dealt round-robin (tile t -> rank t % world, zrt.h); each rank
renders its tiles into a buffer padded to the largest rank's size, and one
gather to the destination rank (RCCL over xGMI with the "nccl" backend; gloo
in the CPU tests) collects them.  The gathered, un-padded buffer is rank-major,
which is what zrt_ctx_assemble expects.
"""
from __future__ import annotations

import ctypes as C

from . import _ffi


def tile_counts(params) -> list:
    """Tiles owned by each rank for these params (zrt_ctx_tile_count, host only)."""
    L = _ffi.load()
    out = []
    for r in range(params.world_size):
        p = params.abi()
        p.rank = r
        n = C.c_uint32()
        _ffi.check(L.zrt_ctx_tile_count(None, C.byref(p), C.byref(n)))
        out.append(n.value)
    return out


def gather_tiles(tiles, counts, rank, world, dst=0, group=None):
    """Gather every rank's padded tile buffer to `dst`; returns the rank-major,
    un-padded concatenation on `dst` and None elsewhere."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return tiles[: counts[0] * 64 * 3]
    send = tiles
    if tiles.is_cuda and dist.get_backend(group) == "gloo":
        send = tiles.cpu()  # gloo gathers host tensors (multi-rank rehearsal on one GPU)
    bufs = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, bufs, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([b[: c * 64 * 3] for b, c in zip(bufs, counts)]).to(tiles.device)
