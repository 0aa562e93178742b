"""Multi-process CPU test (gloo, world size 2) of the frame-sharding path bench.py
runs on N GPUs: tile-cyclic ownership, per-rank packing, ONE gather to rank 0,
unpack, and the max-over-ranks timing reduction.  The GPU pack/unpack kernels
implement the same mapping (checked on the GPU in test_gpu_parity.py)."""
import os
import time
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def synthetic_frame(w, h):
    y, x = np.mgrid[0:h, 0:w]
    return ((x * 2654435761 + y * 40503 + 12345) & 0xFFFFFFFF).astype(np.uint32)


def _worker(rank, world, port, w, h, q):
    import torch
    import torch.distributed as dist

    from gpgpuraytrace_amd import parallel as P
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = synthetic_frame(w, h)
        # each rank "renders" only its tiles
        mine = np.zeros_like(full)
        P.unpack_host(mine, P.pack_host(full, rank, world), rank, world)
        maxb = max(P.shard_bytes(w, h, r, world) for r in range(world))
        packed = np.zeros(maxb // 4, np.uint32)
        pk = P.pack_host(mine, rank, world)
        packed[:pk.size] = pk
        t = torch.from_numpy(packed.view(np.int32).copy())
        frame0 = mine.copy()

        def unpack(src, buf):
            n = P.shard_bytes(w, h, src, world) // 4
            P.unpack_host(frame0, buf.numpy().view(np.uint32)[:n], src, world)

        P.gather_frame(dist, t, w, h, rank, world, unpack)
        el = torch.tensor([0.5 + rank], dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        if rank == 0:
            q.put((bool(np.array_equal(frame0, full)), float(el.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("w,h", [(96, 70), (1920, 1080)])
def test_gloo_two_rank_frame_gather(w, h):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, w, h, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, t = q.get(timeout=10)
    assert ok
    assert t == 1.5  # max over ranks


# --- bench.py's batch sequence (parallel.BatchPlan + run_batch) with host ops ---------------
def synthetic_cameras(f):
    """Stand-in CameraResults of frame f (what the prepass would write)."""
    return (np.arange(1024 * 4, dtype=np.float32) * 0.25 + np.float32(f * 1000.0)).astype(np.float32)


def synthetic_batch_frame(w, h, f, cams):
    """Stand-in for frame f's render: depends on f and on frame f's CameraResults, so a wrong
    all-gather or a wrong frame-to-slot mapping changes the pixels."""
    return synthetic_frame(w, h) ^ np.uint32(f * 0x9E3779B1 & 0xFFFFFFFF) ^ cams.view(np.uint32)[f % 4096]


class HostOps:
    """run_batch's actions with numpy buffers and gloo collectives: the prepass writes the
    stand-in CameraResults of its frames, the trace renders ONLY this rank's rotated shard of
    every frame (other tiles stay zero), pack / unpack use parallel.pack_host / unpack_host."""

    def __init__(self, plan, rank, coll, w, h, n, group=None):
        import torch
        self.p, self.rank, self.coll, self.w, self.h, self.n, self.group = plan, rank, coll, w, h, n, group
        self.cams = torch.full((plan.camera_floats(),), float("nan"), dtype=torch.float32)
        self.frames = [np.zeros((h, w), np.uint32) for _ in range(n)]
        self.packed = torch.zeros(plan.packed_bytes() // 4, dtype=torch.int32)
        self.gathered = [torch.zeros_like(self.packed) for _ in range(plan.world)] if rank == 0 else None
        self.log = []

    def prepass(self, first, count):
        import torch
        self.log.append(("prepass", first, count))
        base = self.p.camera_slice(self.rank).start
        assert base == first * 4096 or count == 0  # the rank's slice holds its own frames
        for i in range(count):
            self.cams[base + i * 4096:base + (i + 1) * 4096] = torch.from_numpy(synthetic_cameras(first + i))

    def all_gather_cameras(self):
        self.coll.all_gather(self.cams, self.cams[self.p.camera_slice(self.rank)].clone(), self.group)

    def _render(self, f, cams):
        from gpgpuraytrace_amd import parallel as P
        full = synthetic_batch_frame(self.w, self.h, f, cams)
        shard = P.frame_shard(self.rank, f, self.p.world)
        P.unpack_host(self.frames[f], P.pack_host(full, shard, self.p.world), shard, self.p.world)

    def trace(self):
        self.log.append(("trace",))
        c = self.cams.numpy()
        for f in range(self.n):
            got = c[f * 4096:(f + 1) * 4096]
            assert np.array_equal(got, synthetic_cameras(f)), f"frame {f}: CameraResults not gathered"
            self._render(f, got)

    def render(self):
        self.log.append(("render",))
        for f in range(self.n):
            self._render(f, synthetic_cameras(f))

    def render_packed(self, items):
        """plan.direct_pack: this rank's shards straight into the packed buffer (the framebuffers stay
        untouched, as on the GPU)."""
        import torch

        from gpgpuraytrace_amd import parallel as P
        self.log.append(("render_packed", len(items)))
        for f, shard, off in items:
            pk = P.pack_host(synthetic_batch_frame(self.w, self.h, f, synthetic_cameras(f)), shard,
                             self.p.world).view(np.int32)
            self.packed[off // 4:off // 4 + pk.size] = torch.from_numpy(pk.copy())

    def prepass_ahead(self):
        self.log.append(("prepass_ahead",))

    def prepass_ahead_next(self):
        self.log.append(("prepass_ahead_next",))

    def trace_ahead(self):
        self.log.append(("trace_ahead",))
        for f in range(self.n):
            self._render(f, synthetic_cameras(f))

    def pack(self, f, shard, off):
        import torch

        from gpgpuraytrace_amd import parallel as P
        pk = P.pack_host(self.frames[f], shard, self.p.world).view(np.int32)
        self.packed[off // 4:off // 4 + pk.size] = torch.from_numpy(pk.copy())

    def pack_batch(self, items):
        self.log.append(("pack_batch", len(items)))
        for f, shard, off in items:
            self.pack(f, shard, off)

    def gather(self):
        self.coll.gather(self.packed, self.gathered)

    def unpack(self, src, f, shard, off):
        from gpgpuraytrace_amd import parallel as P
        n = P.shard_bytes(self.w, self.h, shard, self.p.world) // 4
        buf = self.gathered[src].numpy().view(np.uint32)[off // 4:off // 4 + n]
        P.unpack_host(self.frames[f], buf, shard, self.p.world)

    def unpack_batch(self, items):
        self.log.append(("unpack_batch", len(items)))
        for src, f, shard, off in items:
            self.unpack(src, f, shard, off)

    def present(self):
        self.log.append(("present",))


def _batch_worker(rank, world, port, w, h, batch, frames, split, q):
    import torch.distributed as dist

    from gpgpuraytrace_amd import parallel as P
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        plan = P.BatchPlan(w, h, batch, world, split_prepass=split is True, lookahead=split == "ahead",
                           direct_pack=split == "direct")
        coll = P.Collectives(dist, "gloo", rank, world)
        group = dist.new_group(backend="gloo") if plan.split_prepass else None
        ops = HostOps(plan, rank, coll, w, h, frames, group)
        # bench.py's per-rank phase report, with host clocks in place of HIP events
        dist.barrier()
        t0 = time.perf_counter()
        marks = []
        P.run_batch(plan, rank, ops, frames=frames, mark=lambda name: marks.append((name, time.perf_counter())))
        phases = P.phase_summary([marks], lambda a, b: (b - a) * 1e3, t0=t0)
        phases["rank"] = rank
        per_rank = [None] * world
        dist.all_gather_object(per_rank, phases)
        if rank == 0:
            ok = all(np.array_equal(ops.frames[f], synthetic_batch_frame(w, h, f, synthetic_cameras(f)))
                     for f in range(frames))
            q.put((ok, ops.log, per_rank, P.start_skew(per_rank)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,w,h,batch,frames,split", [
    (2, 1920, 1080, 12, 12, True),   # bench default at N=2
    (3, 1920, 1080, 12, 12, True),   # 2040 tiles % 3 == 0, chunk 4
    (3, 96, 70, 12, 10, True),       # 9 tiles: ragged shards (3 each), partial batch of 10
    (2, 64, 48, 5, 5, True),         # 4 tiles; chunk 3: rank 1 runs 2 prepass frames
    (3, 64, 48, 3, 3, True),         # 4 tiles % 3 != 0: shards of 2, 1, 1 tiles
    (3, 50, 36, 12, 7, False),       # unsplit prepass, partial batch
    (2, 1920, 1080, 12, 12, "ahead"),  # bench default: unsplit, the next batch's prepass queued ahead
    (3, 50, 36, 12, 7, "ahead"),     # the same, partial batch
    (2, 1920, 1080, 12, 12, "direct"),  # bench default (ABI 7): shards rendered straight into the packed buffer
    (3, 50, 36, 12, 7, "direct"),    # the same, ragged shards, partial batch
])
def test_gloo_batch_plan_assembles_frames(world, w, h, batch, frames, split):
    """bench.py's N>1 batch sequence, driven through parallel.run_batch with host ops: split
    prepass chunks + CameraResults all-gather, per-frame shard rotation (r + f) % N, packed
    offsets, one gather, unpack order.  Rank 0 must assemble every frame of the batch."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_batch_worker, args=(r, world, port, w, h, batch, frames, split, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, log, per_rank, skew = q.get(timeout=10)
    assert ok
    from gpgpuraytrace_amd import parallel as P
    plan = P.BatchPlan(w, h, batch, world, split_prepass=split is True, lookahead=split == "ahead",
                       direct_pack=split == "direct")
    if plan.split_prepass:
        assert log[0] == ("prepass", 0, min(plan.chunk, frames)) and ("trace",) in log
    elif plan.lookahead:
        # this batch's prepass, then the next one's, both queued before this trace
        assert log[:3] == [("prepass_ahead",), ("prepass_ahead_next",), ("trace_ahead",)]
    else:
        assert log[0] == ("render",)  # (rank 0 renders into its framebuffers also with direct_pack)
    # rank 0: one pack of its frames (none with direct_pack: its own shards are never sent), one unpack of
    # every other rank's (one launch each on the GPU)
    assert (("pack_batch", frames) in log) != plan.direct_pack and ("unpack_batch", (world - 1) * frames) in log
    # bench.py's config.per_rank / trace_start_skew_ms (make the first 8-GPU run diagnosable)
    assert [r["rank"] for r in per_rank] == list(range(world))
    want = (["prepass", "all_gather"] if plan.split_prepass else []) + ["trace"] + \
        ([] if plan.direct_pack else ["pack"]) + ["gather"]
    for r in per_rank:
        keys = want + (["unpack"] if r["rank"] == 0 else [])
        assert sorted(r["phase_ms"]) == sorted(keys) and sorted(r["phase_ms_max"]) == sorted(keys)
        assert all(v >= 0.0 for v in r["phase_ms"].values()) and r["batches"] == 1
        assert len(r["trace_start_ms"]) == 1 and r["trace_start_ms"][0] >= 0.0
    assert len(skew) == 1 and skew[0] >= 0.0


def test_batch_plan_bookkeeping():
    from gpgpuraytrace_amd import parallel as P
    p = P.BatchPlan(1920, 1080, 12, 8)
    assert p.chunk == 2
    assert [p.prepass_range(r) for r in range(8)] == [(0, 2), (2, 2), (4, 2), (6, 2), (8, 2), (10, 2), (12, 0),
                                                      (12, 0)]
    assert [p.shard(3, f) for f in range(12)] == [(3 + f) % 8 for f in range(12)]
    # every (frame, shard) pair is delivered exactly once: rank 0 packs its own, unpacks the rest
    seen = {(f, s) for f, s, _ in p.packs(0)} | {(f, s) for _, f, s, _ in p.unpacks()}
    assert seen == {(f, s) for f in range(12) for s in range(8)}
    assert p.max_bytes == max(P.shard_bytes(1920, 1080, r, 8) for r in range(8))
    assert P.BatchPlan(64, 48, 3, 3).max_bytes == 2 * 32 * 32 * 4  # shards of 2, 1, 1 tiles
    assert P.frame_shard(5, 0, 1) == 0
    with pytest.raises(ValueError):
        P.BatchPlan(64, 48, 25, 2)  # RT_MAX_BATCH 24 (ABI 6)
    big = P.BatchPlan(1920, 1080, 24, 8)  # the largest batch: every (frame, shard) pair still once
    seen = {(f, s) for f, s, _ in big.packs(0)} | {(f, s) for _, f, s, _ in big.unpacks()}
    assert seen == {(f, s) for f in range(24) for s in range(8)}


def test_phase_summary_leaves_out_unreadable_pairs():
    """bench.py's event_ms returns None when HIP refuses an event pair: that phase (or the trace
    start) is left out of config.per_rank instead of ending the run."""
    from gpgpuraytrace_amd import parallel as P
    marks = [("start", 0.0), ("trace", 2.0), ("pack", 2.5), ("gather", 3.0)]

    def ms(a, b):
        return None if (a, b) == (2.0, 2.5) else b - a

    out = P.phase_summary([marks, marks], ms, t0=0.0)
    assert out["phase_ms"] == {"trace": 2.0, "gather": 0.5}
    assert "pack" not in out["phase_ms_max"]
    assert out["trace_start_ms"] == [0.0, 0.0]
    out = P.phase_summary([marks], lambda a, b: None, t0=0.0)
    assert out["phase_ms"] == {} and out["trace_start_ms"] == []
