"""Multi-GPU plumbing for the tile partition.

8x8 tiles are dealt round-robin (tile t -> rank t % world, zrt.h); each rank
renders its tiles into a buffer padded to the largest rank's size, and one
gather to the destination rank (RCCL over xGMI with the "nccl" backend; gloo
in the CPU tests) collects them straight into one padded, rank-major buffer
(rank r at tile r * max_tiles), which zrt_ctx_assemble_padded reads as it
lies: no un-padding copy.
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


def gather_tiles(tiles, counts, rank, world, dst=0, group=None, out=None):
    """Gather every rank's padded tile buffer (max(counts) tiles) to `dst`.

    Returns, on `dst`, the padded rank-major buffer: rank r's tiles at
    r * max(counts) * 64 * 3 floats (`out` if given, on the device of `tiles`);
    None on the other ranks.  With the nccl backend the per-rank receive
    buffers are views into that one buffer, so RCCL writes each rank's tiles
    in place; gloo (CPU rehearsal, ranks may share a GPU) gathers host copies
    and moves the whole buffer to the device once."""
    import torch
    import torch.distributed as dist
    per_rank = max(counts) * 64 * 3
    if tiles.numel() < per_rank:
        raise ValueError(f"tile buffer holds {tiles.numel()} floats, the padded gather needs {per_rank}")
    send = tiles[:per_rank]
    if world == 1:
        if out is not None:
            out[:per_rank].copy_(send)
            return out
        return send
    gloo = dist.get_backend(group) == "gloo"
    if gloo and send.is_cuda:
        send = send.cpu()  # gloo gathers host tensors
    bufs = None
    if rank == dst:
        if gloo:
            host = torch.empty(world * per_rank, dtype=send.dtype)
            bufs = [host[r * per_rank:(r + 1) * per_rank] for r in range(world)]
        else:
            if out is None:
                out = torch.empty(world * per_rank, dtype=tiles.dtype, device=tiles.device)
            bufs = [out[r * per_rank:(r + 1) * per_rank] for r in range(world)]
    dist.gather(send, bufs, dst=dst, group=group)
    if rank != dst:
        return None
    if gloo:
        if out is None:
            return host.to(tiles.device)
        out[: world * per_rank].copy_(host)
    return out


class TileFrame:
    """One frame of the tile partition on this rank, as bench.py times it:
    render this rank's tiles (scene resident in HBM), gather all ranks' tiles
    to rank 0 (RCCL over xGMI, or gloo), assemble the framebuffer on rank 0.

    Everything is enqueued on one explicit torch stream whose handle is passed
    to libzrt, so the gather (which torch orders after the current stream) and
    the assemble see the finalized tiles, with no reliance on libzrt's own
    stream.  The buffers are allocated once and reused every step."""

    def __init__(self, scene, params, rank: int, world: int):
        import torch
        from . import RenderContext, RenderParams
        self.scene, self.params, self.rank, self.world = scene, params, rank, world
        self.ctx = RenderContext(scene, params)
        self.counts = tile_counts(params)
        self.max_tiles = max(self.counts)
        dev = torch.device("cuda", params.device)
        self.stream = torch.cuda.Stream(device=dev)
        self.tiles = torch.zeros(max(1, self.max_tiles) * 64 * 3, dtype=torch.float32, device=dev)
        self.gathered = self.frame = None
        if rank == 0:
            self.gathered = torch.empty(world * max(1, self.max_tiles) * 64 * 3, dtype=torch.float32, device=dev)
            self.frame = torch.empty(params.height * params.width * 3, dtype=torch.float32, device=dev)
        self.p0 = RenderParams(**{**params.__dict__, "rank": 0})
        self.gather_ms = []  # per step: the gather (+ assemble on rank 0), HIP events on self.stream
        self._ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))

    def step(self, params=None, record: bool = None) -> float:
        """One frame; returns the render launch's kernel time in ms (HIP events
        on the launch stream).  `params` overrides the render params (e.g. the
        diagnostic flag) for this step.  The gather (+ assemble) time is appended
        to gather_ms when `record` is true - by default for steps with the
        frame's own params, so an extra diagnostic launch does not count."""
        import torch
        p = params or self.params
        with torch.cuda.stream(self.stream):
            self.ctx.render_tiles(self.scene.camera, p, self.tiles.data_ptr(), self.stream.cuda_stream)
            kms = self.ctx.kernel_ms()
            self._ev[0].record(self.stream)
            g = gather_tiles(self.tiles, self.counts, self.rank, self.world, dst=0, out=self.gathered)
            if self.rank == 0:
                self.ctx.assemble_padded(self.p0, g.data_ptr(), max(1, self.max_tiles), self.frame.data_ptr(),
                                         self.stream.cuda_stream)
            self._ev[1].record(self.stream)
        if record or (record is None and params is None):
            self._ev[1].synchronize()
            self.gather_ms.append(self._ev[0].elapsed_time(self._ev[1]))
        return kms

    def image(self):
        """Rank 0: the assembled framebuffer as numpy [H, W, 3] (row 0 = bottom)."""
        self.stream.synchronize()
        return self.frame.cpu().numpy().reshape(self.params.height, self.params.width, 3)

    def close(self):
        self.ctx.close()
