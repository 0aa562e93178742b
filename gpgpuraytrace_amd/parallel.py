"""Frame sharding across GPUs (one process per GPU, torch.distributed over RCCL).

The reference renders on one D3D11 adapter (Terrain.cpp:105-136 dispatches the frame's
tiles on it).  Here a frame is split tile-cyclically: 32x32-pixel tiles in row-major order;
shard s of N is the tiles t with t % N == s.  Cyclic dealing balances the ~10x cost spread
between sky and terrain tiles.

bench.py renders BATCHES of B frames (rt_terrain_render_batch) and rotates the shards over a
batch: frame f of rank r's batch traces shard (r + f) % N, so every rank's batch mixes every
shard's tile classes.  BatchPlan holds that bookkeeping and run_batch() is the one sequence of
steps every rank runs per batch; bench.py drives it with device ops (HIP kernels, RCCL) and
tests/test_dist.py with host ops (numpy, gloo), so the CPU tests exercise the same code:

  1. prepass: unsplit (default): every rank runs every frame's camerarays prepass (SURVEY.md
     section 8e's per-rank recompute; 1024 rays a frame).  With lookahead (bench.py
     --lookahead 1) the NEXT batch's prepass is queued on the GPU's side stream before this
     batch's trace (rt_terrain_prepass_ahead) instead of in line on its own slot group's
     stream (DESIGN.md section 7 has the measurements).  Split
     (split_prepass=True): rank r runs the prepass of frames [r*chunk, (r+1)*chunk), chunk =
     ceil(B/N) (ranks past the last frame run an empty range), and an all-gather hands every
     rank all B frames' CameraResults (16 KiB per frame) -- a second collective per batch,
     which the barrier model of DESIGN.md section 7 found slower than recompute.
  2. trace: each rank traces its shard of every frame (setTargetDepths + tracescreen).
  3. pack: frame f's shard (r + f) % N goes to packed[f * max_bytes : ...] (k_shard_copy;
     1024 RGBA8 pixels per tile, tiles in ascending order), the batch's frames in one launch.
     With direct_pack (bench.py's default, the unsplit in-line path) there is no pack step: ranks
     r > 0 render their shards straight into that buffer (rt_terrain_render_batch_packed: the trace
     kernels store each pixel at its packed offset), and rank 0, whose own shards are never sent,
     renders into its framebuffers.  The pack launch used to queue behind the other batch's
     persistent trace kernel before the gather could start.
  4. ONE gather of the packed buffers to rank 0, which unpacks rank src's frame f as shard
     (src + f) % N from gathered[src][f * max_bytes : ...], all (N-1) x B in one launch.

The tile mapping is the one the HIP kernels use (rt_kernels.h rt_shard_tiles, k_shard_copy).
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


def frame_shard(rank, f, world):
    """The shard frame f of a batch traces on `rank` (per-frame rotation; rt_kernels.h
    rt_launch_tracescreen).  A single frame (f = 0) traces shard `rank`."""
    return (rank + f) % world if world > 1 else 0


class BatchPlan:
    """Bookkeeping of one B-frame batch on `world` ranks (see the module docstring)."""

    CAMERA_FLOATS = 1024 * 4  # CameraResults of one frame: float4[1024]

    def __init__(self, width, height, batch, world, split_prepass=False, lookahead=False, direct_pack=False):
        if not 1 <= batch <= 24:
            raise ValueError("batch must be 1..24 frames (RT_MAX_BATCH)")
        self.width, self.height, self.batch, self.world = int(width), int(height), int(batch), int(world)
        self.split_prepass = bool(split_prepass) and self.world > 1
        # the ahead prepass is the unsplit one's (the split one is gathered before its trace)
        self.lookahead = bool(lookahead) and not self.split_prepass
        # shards rendered straight into the packed buffer (the in-line render path only)
        self.direct_pack = bool(direct_pack) and self.world > 1 and not self.split_prepass and not self.lookahead
        self.chunk = -(-self.batch // self.world)
        self.max_bytes = max(shard_bytes(self.width, self.height, r, self.world) for r in range(self.world))

    def shard(self, rank, f):
        return frame_shard(rank, f, self.world)

    def prepass_range(self, rank):
        """(first, count) of the frames whose prepass `rank` runs (count may be 0)."""
        first = min(rank * self.chunk, self.batch)
        return first, max(0, min(self.batch - first, self.chunk))

    def camera_slice(self, rank):
        """rank's part of the all-gathered CameraResults buffer (world * chunk frames), in floats."""
        n = self.chunk * self.CAMERA_FLOATS
        return slice(rank * n, (rank + 1) * n)

    def camera_floats(self):
        return self.world * self.chunk * self.CAMERA_FLOATS

    def packed_bytes(self):
        return self.batch * self.max_bytes

    def pack_offset(self, f):
        return f * self.max_bytes

    def packs(self, rank, frames=None):
        """[(f, shard, byte offset)] this rank packs, frame order."""
        n = self.batch if frames is None else frames
        return [(f, self.shard(rank, f), self.pack_offset(f)) for f in range(n)]

    def unpacks(self, frames=None):
        """[(src rank, f, shard, byte offset in src's gathered buffer)] rank 0 unpacks."""
        n = self.batch if frames is None else frames
        return [(src, f, self.shard(src, f), self.pack_offset(f)) for src in range(1, self.world) for f in range(n)]


def run_batch(plan, rank, ops, frames=None, mark=None, ahead_next=True):
    """One batch on this rank.  `ops` supplies the actions (bench.py: HIP + RCCL; tests: numpy
    + gloo): prepass(first, count), all_gather_cameras(), trace(), render() (prepass + trace of
    every frame, the unsplit path), with plan.lookahead prepass_ahead() (this batch's prepass on
    the side stream, unless the previous batch queued it), prepass_ahead_next() (the next
    batch's, before this trace; skipped with ahead_next=False: the last batch of a run) and
    trace_ahead(), pack_batch([(f, shard, offset)]) (this rank's frames; one
    rt_shard_pack_batch launch on the GPU), with plan.direct_pack render_packed([(f, shard, offset)])
    in place of render() + pack_batch() on ranks > 0 (rank 0 renders and packs nothing: its own
    shards are never sent), gather(), unpack_batch([(src, f, shard, offset)])
    (rank 0: every other rank's frames in one rt_shard_unpack_batch launch), present().
    `frames` < plan.batch renders a partial batch (its first frames).
    mark(name), if given, is called at the start ("start") and after each phase ("prepass",
    "all_gather", "trace", "pack", "gather", "unpack"): bench.py records a HIP event on the
    batch's stream there (PHASES; phase_summary turns the marks into per-phase times)."""
    n = plan.batch if frames is None else int(frames)
    mark = mark or (lambda name: None)
    mark("start")
    if plan.split_prepass:
        first, count = plan.prepass_range(rank)
        count = max(0, min(count, n - first))
        ops.prepass(first, count)
        mark("prepass")
        ops.all_gather_cameras()
        mark("all_gather")
        ops.trace()
    elif plan.lookahead:
        ops.prepass_ahead()
        if ahead_next:
            ops.prepass_ahead_next()
        ops.trace_ahead()
    elif plan.direct_pack and rank > 0:
        ops.render_packed(plan.packs(rank, n))
    else:
        ops.render()
    mark("trace")
    if plan.world > 1:
        if not plan.direct_pack:
            ops.pack_batch(plan.packs(rank, n))
            mark("pack")
        ops.gather()
        mark("gather")
        if rank == 0:
            ops.unpack_batch(plan.unpacks(n))
            mark("unpack")
    ops.present()


PHASES = ("prepass", "all_gather", "trace", "pack", "gather", "unpack")


def phase_summary(batches, elapsed_ms, t0=None):
    """Per-phase times of one rank's batches.  batches: per batch the [(name, clock)] marks of
    run_batch (a HIP event or a host time); elapsed_ms(a, b): ms from clock a to clock b, or None when unreadable (left out); t0: the
    clock the timed region started at (per batch, or one for all), for each batch's trace start.
    Returns {"batches", "phase_ms" (mean per batch), "phase_ms_max", "trace_start_ms" (per batch,
    from t0: the prepass + all-gather end; the batch start when the prepass is not split)}.  A
    phase's time is from the previous mark: it includes any wait of the batch's stream for the
    other batch in flight (the co-scheduling DESIGN.md section 7 describes)."""
    per = {p: [] for p in PHASES}
    starts = []
    for i, marks in enumerate(batches):
        for (_, a), (name, b) in zip(marks, marks[1:]):
            ms = elapsed_ms(a, b)
            if ms is not None:  # None: the clock pair could not be read (the phase is left out)
                per[name].append(ms)
        if t0 is not None:
            z = t0[i] if isinstance(t0, (list, tuple)) else t0
            names = [m[0] for m in marks]
            at = marks[names.index("all_gather")][1] if "all_gather" in names else marks[0][1]
            ms = elapsed_ms(z, at)
            if ms is not None:
                starts.append(ms)
    out = {"batches": len(batches),
           "phase_ms": {p: round(float(sum(v) / len(v)), 4) for p, v in per.items() if v},
           "phase_ms_max": {p: round(float(max(v)), 4) for p, v in per.items() if v}}
    if t0 is not None:
        out["trace_start_ms"] = [round(float(x), 4) for x in starts]
    return out


def start_skew(per_rank):
    """Per batch: the spread (max - min over ranks) of the trace start, from the ranks'
    phase_summary()s (their t0 is the common barrier that starts the timed region)."""
    starts = [r["trace_start_ms"] for r in per_rank if "trace_start_ms" in r]
    if not starts:
        return []
    return [round(max(c) - min(c), 4) for c in zip(*starts)]


class Collectives:
    """The two collectives of run_batch over torch.distributed: device-memory RCCL
    (backend "nccl") or host-staged gloo (rehearsals on one GPU, CPU tests)."""

    def __init__(self, dist, backend, rank, world):
        self.dist, self.backend, self.rank, self.world = dist, backend, rank, world

    def all_gather(self, out, mine, group=None):
        if self.backend == "nccl":
            self.dist.all_gather_into_tensor(out, mine, group=group)
            return
        import torch
        parts = [torch.empty(mine.numel(), dtype=mine.dtype) for _ in range(self.world)]
        self.dist.all_gather(parts, mine.cpu(), group=group)
        out.copy_(torch.cat(parts).to(out.device))

    def gather(self, t, outs):
        """t from every rank into outs[src] on rank 0 (outs ignored elsewhere)."""
        if self.backend == "nccl":
            self.dist.gather(t, outs if self.rank == 0 else None, dst=0)
            return
        import torch
        lst = [torch.empty(t.numel(), dtype=t.dtype) for _ in range(self.world)] if self.rank == 0 else None
        self.dist.gather(t.cpu(), lst, dst=0)
        if self.rank == 0:
            for o, part in zip(outs, lst):
                o.copy_(part.to(o.device))
