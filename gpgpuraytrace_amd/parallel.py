"""Frame sharding across GPUs (one process per GPU, torch.distributed over RCCL).

The reference renders on one D3D11 adapter.  Here a frame is split tile-cyclically:
32x32-pixel tiles in row-major order, tile t belongs to rank t % world.  Every rank
recomputes the 1024-ray prepass (tiny, deterministic) so no collective precedes the
trace; afterwards each rank packs its tiles (1024 pixels per tile, RGBA8) and ONE
gather assembles the frame on rank 0.  Cyclic dealing balances the ~10x cost spread
between sky and terrain tiles.

The mapping here is the same one the HIP kernels use (rt_kernels.h rt_shard_tiles,
k_shard_copy); the host functions are used by the CPU (gloo) tests.
"""
import numpy as np

TILE = 32


def tiles_xy(width, height):
    return (width + TILE - 1) // TILE, (height + TILE - 1) // TILE


def shard_tiles(width, height, rank, world):
    """Tile indices owned by `rank` (t % world == rank), in packing order."""
    tx, ty = tiles_xy(width, height)
    return np.arange(rank, tx * ty, world, dtype=np.int64)


def shard_bytes(width, height, rank, world):
    return len(shard_tiles(width, height, rank, world)) * TILE * TILE * 4


def pack_host(frame, rank, world):
    """frame: (H, W) uint32 (RGBA8) -> packed uint32 array of this rank's tiles (k_shard_copy, pack)."""
    h, w = frame.shape
    tx, _ = tiles_xy(w, h)
    tiles = shard_tiles(w, h, rank, world)
    out = np.zeros((len(tiles), TILE * TILE), np.uint32)
    for k, t in enumerate(tiles):
        x0, y0 = (t % tx) * TILE, (t // tx) * TILE
        blk = frame[y0:y0 + TILE, x0:x0 + TILE]
        tmp = np.zeros((TILE, TILE), np.uint32)
        tmp[:blk.shape[0], :blk.shape[1]] = blk
        out[k] = tmp.ravel()
    return out.ravel()


def unpack_host(frame, packed, rank, world):
    """Inverse of pack_host into `frame` (k_shard_copy, unpack)."""
    h, w = frame.shape
    tx, _ = tiles_xy(w, h)
    tiles = shard_tiles(w, h, rank, world)
    p = packed.reshape(-1, TILE * TILE)
    for k, t in enumerate(tiles):
        x0, y0 = (t % tx) * TILE, (t // tx) * TILE
        blk = p[k].reshape(TILE, TILE)
        hh, ww = min(TILE, h - y0), min(TILE, w - x0)
        frame[y0:y0 + hh, x0:x0 + ww] = blk[:hh, :ww]
    return frame


def gather_frame(dist, packed, width, height, rank, world, unpack):
    """Gather every rank's packed tile buffer (a torch tensor of max-shard size) on rank 0
    and hand each one to `unpack(src_rank, tensor)`.  One collective per frame."""
    import torch
    bufs = [torch.empty_like(packed) for _ in range(world)] if rank == 0 else None
    dist.gather(packed, bufs, dst=0)
    if rank == 0:
        for r in range(1, world):
            unpack(r, bufs[r])
    return bufs
