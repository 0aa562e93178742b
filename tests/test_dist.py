"""Multi-process CPU test (gloo, world size 2) of the frame-sharding path bench.py
runs on N GPUs: tile-cyclic ownership, per-rank packing, ONE gather to rank 0,
unpack, and the max-over-ranks timing reduction.  The GPU pack/unpack kernels
implement the same mapping (checked on the GPU in test_gpu_parity.py)."""
import os
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
