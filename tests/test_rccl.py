"""RCCL (torch.distributed backend "nccl") at world size 1 on one MI355X: every collective call
bench.py makes at N > 1, with the tensors, dtypes and streams it uses there, so the RCCL API path
executes on the GPU box before the driver's multi-GPU run (the multi-rank data movement itself is
covered by the gloo tests of tests/test_dist.py, which drive the same parallel.run_batch).

  * parallel.Collectives.all_gather (all_gather_into_tensor, the split prepass's camera gather)
    and .gather (dist.gather of the packed shard buffers to rank 0), issued under
    torch.cuda.stream(ExternalStream(<a device's HIP stream>)) exactly as bench.py's DeviceOps do,
    followed by a HIP kernel on that same stream (rt_shard_unpack_batch reading the gathered
    buffer), which must see the collective's result;
  * bench.py's barrier, the float64 MAX all-reduce of the elapsed time and all_gather_object of
    the per-rank phase summaries.
"""
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


@pytest.mark.gpu
def test_rccl_world1_collectives_on_batch_stream():
    import torch
    import torch.distributed as dist

    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import engine as E
    from gpgpuraytrace_amd import parallel as P

    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    dev = None
    try:
        assert dist.get_backend() == "nccl"
        W, H = 96, 70
        dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, W, H, gpu=0)
        assert dev is not None
        stream = torch.cuda.ExternalStream(dev.stream(), device="cuda:0")
        coll = P.Collectives(dist, "nccl", 0, 1)

        # the camera all-gather (world * chunk frames of float4[1024]); one rank: out == mine
        plan = P.BatchPlan(W, H, 3, 1)
        cams = torch.zeros(3 * P.BatchPlan.CAMERA_FLOATS, dtype=torch.float32, device="cuda:0")
        mine = torch.arange(cams.numel(), dtype=torch.float32, device="cuda:0")
        torch.cuda.synchronize()  # the fills ran on torch's stream, not on the batch stream
        with torch.cuda.stream(stream):
            coll.all_gather(cams, mine)
        # the packed-shard gather: one uint8 buffer per rank on rank 0
        tx, ty = P.tiles_xy(W, H)
        nbytes = tx * ty * P.TILE * P.TILE * 4
        rng = np.random.default_rng(7)
        frame = rng.integers(0, 2**32, size=(H, W), dtype=np.uint64).astype(np.uint32)
        packed = torch.from_numpy(P.pack_host(frame, 0, 1).view(np.uint8).copy()).to("cuda:0")
        assert packed.numel() == nbytes
        gathered = [torch.zeros(nbytes, dtype=torch.uint8, device="cuda:0")]
        torch.cuda.synchronize()  # the fills ran on torch's stream, not on the batch stream
        with torch.cuda.stream(stream):
            coll.gather(packed, gathered)
        # a HIP kernel on the batch stream reads the gathered buffer: rt_shard_unpack_batch of
        # shard 0 of 1 rebuilds the whole frame on the device
        E.shard_unpack_batch([dev], [0], 1, [gathered[0].data_ptr()])
        dev.synchronize()
        assert torch.equal(cams.cpu(), mine.cpu())
        got = dev.readback()
        assert np.array_equal(got.view(np.uint32).reshape(H, W), frame)

        # bench.py's timing reductions
        dist.barrier()
        t = torch.tensor([1.25, 7.5], dtype=torch.float64, device="cuda:0")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        assert t.cpu().tolist() == [1.25, 7.5]
        per_rank = [None]
        dist.all_gather_object(per_rank, {"phase_ms": {"trace": 1.0}})
        assert per_rank == [{"phase_ms": {"trace": 1.0}}]
    finally:
        if dev is not None:
            dev.destroy()
        dist.destroy_process_group()
